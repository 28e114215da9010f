#!/bin/bash
# Same-box A/B of experiment libraries (tools/exp_lib.sh): for each name ("default" = the
# product build) the 1M-hex8 linear evaluate (tools/eval_timing.py) and, with TSI=1, the fused
# TSI pass (tools/tsi_bench.py), alternated over two rounds.  usage: tools/exp_ab.sh name...
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
for rep in $(seq ${ROUNDS:-2}); do
  for v in "$@"; do
    if [ "$v" = default ]; then unset FCG_LIB; else export FCG_LIB=$v; fi
    if [ -z "$NOLIN" ]; then
      r=$(timeout -k 10 120 python tools/eval_timing.py --n 100 --reps 60 | tail -1) || exit 1
      echo "$v linear $(echo "$r" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(round(d["ms_evaluate"],4))')"
    fi
    if [ -n "$TSI" ]; then
      r=$(timeout -k 10 180 python tools/tsi_bench.py --reps 20 | tail -1) || exit 1
      echo "$v tsi_fused $(echo "$r" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(round(d["ms_fused"],4))')"
    fi
  done
done
