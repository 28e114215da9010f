#!/bin/bash
# round 4, call 22: implicit 2:1 box transfers -- tests, config-3 Newton A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_multigrid.py tests/test_tangent_apply.py \
  > $O/call22_tests.log 2>&1; rc=$?
tail -n 5 $O/call22_tests.log
[ $rc -eq 0 ] || exit $rc
for bt in 1 0; do
  FCG_MG_BOXT=$bt timeout -k 10 500 python tools/newton_bench.py --celltype hex27 --kinem totlag --n 100 --length 1 --load -1 --mg --mg-matrix-free \
    > $O/newton27_b$bt.json 2> $O/newton27_b$bt.err || exit 1
  python -c "import json; d=json.loads(open('$O/newton27_b$bt.json').read().strip().splitlines()[-1]); print('boxt=$bt', {k: d[k] for k in ('newton_s','solve_ms_total','pcg_iterations','tip_uz')})"
done
