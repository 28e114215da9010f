#!/bin/bash
# round 4, call 5: gather record order A/B + parity, gather traffic, primary-line kernel statistics
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gather_tiled.py -k "gather or renumbered or lattice" 2>&1 | tail -3 || exit 1
for rep in 1 2; do for v in default gcont; do for k in linear totlag; do
  if [ "$v" = default ]; then unset FCG_LIB; else export FCG_LIB=$v; fi
  r=$(timeout -k 10 200 python tools/eval_timing.py --n 100 --kinem $k --renumber --path gather --reps 30 | tail -1) || exit 1
  echo "$v gather_$k $(echo "$r" | python3 -c 'import json,sys; print(round(json.load(sys.stdin)["ms_evaluate"],4))')" | tee -a $O/ab_gather_rr.txt
done; done; done
unset FCG_LIB
bash tools/pmc_kernel.sh r04/gather_rr "gather_h8_kernel<0, true, true, false>" mem -- --n 100 --path gather --renumber --reps 3 > $O/gather_rr_pmc.log 2>&1 || exit 1
tail -4 $O/gather_rr/summary.txt
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/prim2" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --only-primary --steps 20 --warmup 5) > $O/prim2_bench.json 2> $O/prim2_bench.err || exit 1
tail -c 300 $O/prim2_bench.json
find $O/prim2 -name "*kernel_stats.csv" | head -3
