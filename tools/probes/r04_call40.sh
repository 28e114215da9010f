#!/bin/bash
# round 4, call 40: lanes per block row of the 6 x 6 BSR SpMV (native AMG coarse levels), AMG Newton A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r04
mkdir -p $O
NB="tools/newton_bench.py --celltype hex8 --kinem totlag --n 100 --length 1 --load=-1e-2 --renumber --amg-native"
for r in 1 2; do
  for l in 8 16 32; do
    FCG_BSR_LPN66=$l timeout -k 10 240 python3 $NB > $O/amg_lpn66_$l.json 2> $O/amg_lpn66_$l.err || exit 1
    python3 -c "
import json; d=json.loads(open('$O/amg_lpn66_$l.json').read().splitlines()[-1])
print('lpn $l', 'newton_s', round(d['newton_s'],3), 'solve_ms', round(d['solve_ms_total'],1), 'iters', d['pcg_iterations'])
" | tee -a $O/lpn66_ab.txt
  done
done
