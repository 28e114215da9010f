#!/bin/bash
# round 4, call 39: lanes per block row of the 3 x 3 BSR SpMV (native AMG level 0), AMG Newton A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r04
mkdir -p $O
NB="tools/newton_bench.py --celltype hex8 --kinem totlag --n 100 --length 1 --load=-1e-2 --renumber --amg-native"
for r in 1 2; do
  for l in 8 4 16 32; do
    FCG_BSR_LPN33=$l timeout -k 10 240 python3 $NB > $O/amg_lpn$l.json 2> $O/amg_lpn$l.err || exit 1
    python3 -c "
import json; d=json.loads(open('$O/amg_lpn$l.json').read().splitlines()[-1])
print('lpn $l', 'newton_s', round(d['newton_s'],3), 'solve_ms', round(d['solve_ms_total'],1), 'iters', d['pcg_iterations'])
" | tee -a $O/lpn_ab.txt
  done
done
