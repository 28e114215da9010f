#!/bin/bash
# round 4, call 14: dense coarsest level -- multigrid tests, config-3 Newton A/B (dense vs pcg coarsest), kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r04
mkdir -p $O/newton_stats2
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_multigrid.py tests/test_tangent_apply.py \
  > $O/call14_tests.log 2>&1; rc=$?
tail -n 3 $O/call14_tests.log
[ $rc -eq 0 ] || exit $rc
for c in dense pcg; do
  timeout -k 10 500 python tools/newton_bench.py --celltype hex27 --kinem totlag --n 100 --length 1 --load -1 --mg --mg-matrix-free --mg-coarse $c \
    > $O/newton27_c$c.json 2> $O/newton27_c$c.err || exit 1
  python -c "import json; d=json.loads(open('$O/newton27_c$c.json').read().strip().splitlines()[-1]); print('$c', {k: d[k] for k in ('newton_s','solve_ms_total','pcg_iterations','tip_uz')})"
done
(cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/newton_stats2" -o run -- \
  python3 "$GRAFT_REPO_ROOT/tools/newton_bench.py" --celltype hex27 --kinem totlag --n 100 --length 1 --load -1 --mg --mg-matrix-free) > $O/newton_stats2.log 2>&1 || exit 1
