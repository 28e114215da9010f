#!/bin/bash
# round 4, call 28 (run twice: point GJ, then block GJ): native AMG with the dense coarsest inverse + graph-replayed FCG iteration:
# AMG tests, then the renumbered 1M hex8 TotLag Newton A/B (graph / eager / CG coarse), then a
# kernel-trace of the new default
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r04
mkdir -p $O/amg_stats2
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_amg.py > $O/call28_tests.log 2>&1 || { tail -30 $O/call28_tests.log; exit 1; }
tail -3 $O/call28_tests.log
NB="tools/newton_bench.py --celltype hex8 --kinem totlag --n 100 --length 1 --load=-1e-2 --renumber --amg-native"
FCG_AMG_GRAPH=1 timeout -k 10 240 python3 $NB > $O/amg_ab_graph.json 2> $O/amg_ab_graph.err || exit 1
timeout -k 10 240 python3 $NB > $O/amg_ab_eager.json 2> $O/amg_ab_eager.err || exit 1
FCG_AMG_DENSE=0 timeout -k 10 240 python3 $NB > $O/amg_ab_cg.json 2> $O/amg_ab_cg.err || exit 1
for f in graph eager cg; do python3 -c "
import json; d=json.loads(open('$O/amg_ab_$f.json').read().splitlines()[-1])
print('$f', 'newton_s', round(d['newton_s'],3), 'solve_ms', round(d['solve_ms_total'],1), 'iters', d['pcg_iterations'], 'setup_ms', [round(x,1) for x in d['amg_numeric_setup_ms']], d['amg_stats'])
"; done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/amg_stats2" -o run -- \
  python3 "$GRAFT_REPO_ROOT/tools/newton_bench.py" --celltype hex8 --kinem totlag --n 100 --length 1 --load=-1e-2 --renumber --amg-native) > $O/amg_stats2.log 2>&1 || exit 1
echo done
