#!/bin/bash
# Sweep MODE 3 (deferred lower-plane blocks): parity tests, then 1M hex8 timing native vs
# renumbered with FCG_SWEEP_DEFER 0 / 1 on one box, and the renumbered WRITE_SIZE / FETCH_SIZE.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
TAG=${TAG:-r03_defer}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py -k "defer or lattice or renumbered or structured or gather" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for K in linear totlag; do
    for R in "" "--renumber"; do
      for D in 0 1; do
        FCG_SWEEP_DEFER=$D timeout -k 10 200 python tools/eval_timing.py --n 100 --kinem $K --reps 7 $R \
          | sed "s/^/defer=$D /" >> gpurun_out/${TAG}_timing.txt || exit 1
      done
    done
  done
done
python3 - gpurun_out/${TAG}_timing.txt <<'PY'
import json, sys
for line in open(sys.argv[1]):
    tag = line.split("{")[0].strip(); d = json.loads(line[line.index("{"):])
    print(f"{tag} {d['config']:45s} path {d['path']} {d['ms_evaluate']:.3f} ms")
PY
export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_pmc/p$C" -o run -- \
    python3 "$GRAFT_REPO_ROOT/tools/prof_kernel.py" --n 100 --reps 3 --renumber) > gpurun_out/${TAG}_pmc_$C.log 2>&1
  rc=$?; echo "pmc $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 tools/pmc_summary.py gpurun_out/${TAG}_pmc sweep_h8 | tee gpurun_out/${TAG}_pmc_summary.txt
