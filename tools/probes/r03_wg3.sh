#!/bin/bash
# Third sweep workgroup per CU, timing probe: lib wg3 = launch bound 3 with
# the in-plane hold buffer shared by all columns (48 KB LDS, 168 VGPRs, 13-16 spilled; values
# wrong, timing only), wg2probe = the same LDS cut at the default bound (control).  Same box,
# alternated; the plan's segment rule told 3 workgroups per CU for wg3.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
for rep in 1 2 3; do
  for v in default wg2probe wg3 wg3seg; do
    case $v in
      default) unset FCG_LIB; unset FCG_SWEEP_WGS_PER_CU;;
      wg2probe) export FCG_LIB=wg2probe; unset FCG_SWEEP_WGS_PER_CU;;
      wg3) export FCG_LIB=wg3; unset FCG_SWEEP_WGS_PER_CU;;
      wg3seg) export FCG_LIB=wg3; export FCG_SWEEP_WGS_PER_CU=3;;
    esac
    r=$(timeout -k 10 120 python tools/eval_timing.py --n 100 --reps 60 | tail -1) || exit 1
    echo "$v linear $(echo "$r" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(round(d["ms_evaluate"],4))')"
  done
done
