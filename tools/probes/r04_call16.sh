#!/bin/bash
# round 4, call 16: Chebyshev degree A/B for the matrix-free fine smoother (config-3 Newton)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r04
mkdir -p $O
for nu in 2 3 4; do
  timeout -k 10 500 python tools/newton_bench.py --celltype hex27 --kinem totlag --n 100 --length 1 --load -1 --mg --mg-matrix-free --mg-nu $nu \
    > $O/newton27_nu$nu.json 2> $O/newton27_nu$nu.err || exit 1
  python -c "import json; d=json.loads(open('$O/newton27_nu$nu.json').read().strip().splitlines()[-1]); print('nu=$nu', {k: d[k] for k in ('newton_s','solve_ms_total','pcg_iterations','tip_uz')})"
done
