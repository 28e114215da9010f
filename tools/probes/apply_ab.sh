#!/bin/bash
# Same-box A/B of the matrix-free hex27 action (tools/probes/apply_timing.py) across experiment
# libraries (tools/exp_lib.sh; "default" = the product build), alternated over ROUNDS rounds.
# usage: [N=64] [KIN=totlag] [ROUNDS=2] tools/probes/apply_ab.sh name...
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
for rep in $(seq ${ROUNDS:-2}); do
  for v in "$@"; do
    if [ "$v" = default ]; then unset FCG_LIB; else export FCG_LIB=$v; fi
    r=$(timeout -k 10 240 python3 tools/probes/apply_timing.py --n ${N:-64} --kinem ${KIN:-totlag} --reps 30 | tail -1) || exit 1
    echo "$v ${KIN:-totlag} $(echo "$r" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(round(d["ms_tangent_apply"],4), d["rel_diff"])')"
  done
done
