#!/bin/bash
# round 4, call 36: planned Galerkin products with the C blocks formed by aggregate vs in storage order:
# AMG tests, then the renumbered 1M hex8 TotLag Newton (same box, alternating) and kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r04
mkdir -p $O/amg_stats4
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_amg.py > $O/call36_tests.log 2>&1 || { tail -30 $O/call36_tests.log; exit 1; }
tail -2 $O/call36_tests.log
NB="tools/newton_bench.py --celltype hex8 --kinem totlag --n 100 --length 1 --load=-1e-2 --renumber --amg-native"
for r in 1 2; do
  timeout -k 10 240 python3 $NB > $O/amg_ord_$r.json 2> $O/amg_ord_$r.err || exit 1
  FCG_AMG_PLAN_ORDER=0 timeout -k 10 240 python3 $NB > $O/amg_unord_$r.json 2> $O/amg_unord_$r.err || exit 1
  for f in ord_$r unord_$r; do python3 -c "
import json; d=json.loads(open('$O/amg_$f.json').read().splitlines()[-1])
print('$f', 'newton_s', round(d['newton_s'],3), 'solve_ms', round(d['solve_ms_total'],1), 'iters', d['pcg_iterations'], 'setup_ms', [round(x,1) for x in d['amg_numeric_setup_ms']], 'graph_setup_s', round(d['amg_graph_setup_s'],2), 'tip', repr(d['tip_uz']))
"; done
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/amg_stats4" -o run -- \
  python3 "$GRAFT_REPO_ROOT/tools/newton_bench.py" --celltype hex8 --kinem totlag --n 100 --length 1 --load=-1e-2 --renumber --amg-native) > $O/amg_stats4.log 2>&1 || exit 1
grep -E "spgemm" $O/amg_stats4/run_kernel_stats.csv | cut -c1-200
