#!/bin/bash
# TSI thermal pass: explicit 16-byte reads of the shape values and point records (product build)
# against the paired 8-byte reads (thold); TSI tests on the product build
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r06; mkdir -p $O
PYTEST_SEL="tests/test_tsi.py tests/test_gpu_parity.py" bash tools/probes/r06.sh sel || exit 1
for rep in 1 2 3; do for v in default thold; do
  if [ "$v" = default ]; then unset FCG_LIB; else export FCG_LIB=$v; fi
  r=$(timeout -k 10 200 python3 tools/tsi_bench.py --reps 20 | tail -1) || exit 1
  echo "$v $(echo "$r" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(round(d["ms_fused"],4), round(d["ms_structure"],4))')" | tee -a $O/tsi_th_ab.txt
done; done; unset FCG_LIB
