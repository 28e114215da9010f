#!/bin/bash
# round 4, call 34: the incidence sum of fcg_tangent_apply, unconditional 8-way loads (default)
# vs the loop (FCG_LIB=incloop), 100^3 hex27 TotLag, same box alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r04
mkdir -p $O
for r in 1 2; do
  for v in default incloop; do
    if [ "$v" = default ]; then unset FCG_LIB; else export FCG_LIB=$v; fi
    echo "$v $(timeout -k 10 200 python3 tools/probes/apply_timing.py --n 100 --kinem totlag --reps 30 | tail -1)" | tee -a $O/incsum_ab.txt || exit 1
  done
done
