#!/bin/bash
# round 4, call 31: fused Chebyshev step (fcg_chebyshev_step) -- multigrid tests, then config 3
# full Newton fused vs separate passes (same box, alternating)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_multigrid.py tests/test_tangent_apply.py > $O/call31_tests.log 2>&1 || { tail -30 $O/call31_tests.log; exit 1; }
tail -2 $O/call31_tests.log
NB="tools/newton_bench.py --celltype hex27 --kinem totlag --n 100 --length 1 --load -1 --mg --mg-matrix-free --mg-outer-matrix-free"
for r in 1 2; do
  timeout -k 10 300 python3 $NB > $O/c3_fused_$r.json 2> $O/c3_fused_$r.err || exit 1
  FCG_MG_FUSED=0 timeout -k 10 300 python3 $NB > $O/c3_sep_$r.json 2> $O/c3_sep_$r.err || exit 1
  for f in fused_$r sep_$r; do python3 -c "
import json; d=json.loads(open('$O/c3_$f.json').read().splitlines()[-1])
print('$f', 'newton_s', round(d['newton_s'],3), 'solve_ms', round(d['solve_ms_total'],1), 'iters', d['pcg_iterations'], 'tip', repr(d['tip_uz']), [h['norm_res'] for h in d['history']])
"; done
done
