#!/bin/bash
# hex27 pencil-order direct assembly (FCG_PATH_COLORED, StVK): parity subset, then timing against
# the record + row-assembly path (40^3 TotLag / linear, 100^3 TotLag), then HBM traffic (PMC).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
TAG=${TAG:-r03_pencil_v1}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py -k "27 or colored or singular or negative" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
for p in colored general; do
  for k in totlag linear; do
    timeout -k 10 150 python tools/eval_timing.py --celltype hex27 --kinem $k --n 40 --reps 7 --path $p | sed "s/^/$p /" >> gpurun_out/${TAG}_timing.txt || exit 1
  done
done
timeout -k 10 300 python tools/eval_timing.py --celltype hex27 --kinem totlag --n 100 --reps 5 --path colored | sed "s/^/colored /" >> gpurun_out/${TAG}_timing.txt || exit 1
cat gpurun_out/${TAG}_timing.txt
for C in FETCH_SIZE WRITE_SIZE; do
  (cd /tmp && timeout -k 10 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_pmc/$C" -o run -- \
    python3 "$GRAFT_REPO_ROOT/tools/prof_kernel.py" --celltype hex27 --kinem totlag --n 40 --path colored --reps 3) > gpurun_out/${TAG}_pmc_$C.log 2>&1
  rc=$?; echo "pmc $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
