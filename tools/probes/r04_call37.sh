#!/bin/bash
# round 4, call 37: native AMG with level 0 in Morton order -- AMG / multi-rank / C++ tests, then
# the renumbered 1M hex8 TotLag Newton reordered vs context order (same box, alternating)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r04
mkdir -p $O/amg_stats5
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_amg.py tests/test_multigpu.py tests/test_integration_cxx.py > $O/call37_tests.log 2>&1 || { tail -40 $O/call37_tests.log; exit 1; }
tail -2 $O/call37_tests.log
NB="tools/newton_bench.py --celltype hex8 --kinem totlag --n 100 --length 1 --load=-1e-2 --renumber --amg-native"
for r in 1 2; do
  timeout -k 10 240 python3 $NB > $O/amg_mort_$r.json 2> $O/amg_mort_$r.err || exit 1
  FCG_AMG_REORDER=0 timeout -k 10 240 python3 $NB > $O/amg_ctx_$r.json 2> $O/amg_ctx_$r.err || exit 1
  for f in mort_$r ctx_$r; do python3 -c "
import json; d=json.loads(open('$O/amg_$f.json').read().splitlines()[-1])
print('$f', 'newton_s', round(d['newton_s'],3), 'solve_ms', round(d['solve_ms_total'],1), 'iters', d['pcg_iterations'], 'setup_ms', [round(x,1) for x in d['amg_numeric_setup_ms']], 'graph_setup_s', round(d['amg_graph_setup_s'],2), 'tip', repr(d['tip_uz']), [l['dofs'] for l in d['mg_levels']])
"; done
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/amg_stats5" -o run -- \
  python3 "$GRAFT_REPO_ROOT/tools/newton_bench.py" --celltype hex8 --kinem totlag --n 100 --length 1 --load=-1e-2 --renumber --amg-native) > $O/amg_stats5.log 2>&1 || exit 1
head -8 $O/amg_stats5/run_kernel_stats.csv | cut -c1-160
