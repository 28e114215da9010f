#!/bin/bash
# round 4, call 41: full GPU suite + smoke + default bench at HEAD (v7)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 1500 python -u -m pytest -v --timeout 800 --timeout-method thread -m gpu tests > $O/gpu_tests_v7.log 2>&1; rc=$?
tail -n 5 $O/gpu_tests_v7.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tee $O/smoke_v7.log || exit 1
timeout -k 10 900 python bench.py > $O/bench_v7.json 2> $O/bench_v7.err; rc3=$?
tail -c 400 $O/bench_v7.json
[ $((rc | rc3)) -eq 0 ] || exit $((rc | rc3))
# and the restriction SpMV's lanes per row (FCG_BSR_LPN63: 32 default vs 8), AMG Newton
NB="tools/newton_bench.py --celltype hex8 --kinem totlag --n 100 --length 1 --load=-1e-2 --renumber --amg-native"
for r in 1 2; do
  for l in 32 8; do
    FCG_BSR_LPN63=$l timeout -k 10 240 python3 $NB > $O/amg_lpn63_$l.json 2> $O/amg_lpn63_$l.err || exit 1
    python3 -c "
import json; d=json.loads(open('$O/amg_lpn63_$l.json').read().splitlines()[-1])
print('lpn63 $l', 'newton_s', round(d['newton_s'],3), 'solve_ms', round(d['solve_ms_total'],1), 'iters', d['pcg_iterations'])
" | tee -a $O/lpn63_ab.txt
  done
done
