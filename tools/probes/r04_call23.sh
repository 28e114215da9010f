#!/bin/bash
# round 4, call 23: coarse-level Chebyshev degree and V / W cycle below the fine level (config-3 Newton)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r04
mkdir -p $O
for cfg in "2 V" "4 V" "2 W" "4 W"; do
  set -- $cfg
  FCG_MG_COARSE_NU=$1 FCG_MG_CYCLE=$2 timeout -k 10 500 python tools/newton_bench.py --celltype hex27 --kinem totlag --n 100 --length 1 --load -1 --mg --mg-matrix-free \
    > $O/newton27_c$1$2.json 2> $O/newton27_c$1$2.err || exit 1
  python -c "import json; d=json.loads(open('$O/newton27_c$1$2.json').read().strip().splitlines()[-1]); print('coarse_nu=$1 cycle=$2', {k: d[k] for k in ('newton_s','solve_ms_total','pcg_iterations')})"
done
