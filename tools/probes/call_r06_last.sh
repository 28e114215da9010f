#!/bin/bash
# last call of round 6: TSI thermal-read A/B repeated, full suite, smoke and bench on the product build
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r06; mkdir -p $O
for rep in 1 2 3; do for v in default thold; do
  if [ "$v" = default ]; then unset FCG_LIB; else export FCG_LIB=$v; fi
  r=$(timeout -k 10 200 python3 tools/tsi_bench.py --reps 20 | tail -1) || exit 1
  echo "$v $(echo "$r" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(round(d["ms_fused"],4), round(d["ms_structure"],4))')" | tee -a $O/tsi_th_ab.txt
done; done; unset FCG_LIB
bash tools/probes/r06.sh suite smoke bench || exit 1
