#!/bin/bash
# End of round 6: TSI thermal-pass hold rows (holdth10) A/B + its tests, then the full GPU suite,
# smoke and the driver's default bench on the product build
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r06; mkdir -p $O
FCG_LIB=holdth10 PYTEST_SEL="tests/test_tsi.py" bash tools/probes/r06.sh sel || exit 1
for rep in 1 2 3; do for v in default holdth10; do
  if [ "$v" = default ]; then unset FCG_LIB; else export FCG_LIB=$v; fi
  r=$(timeout -k 10 200 python3 tools/tsi_bench.py --reps 20 | tail -1) || exit 1
  echo "$v $(echo "$r" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(round(d["ms_structure"],4), round(d["ms_tsi_blocks"],4), round(d["ms_two_field_tangent"],4))')" | tee -a $O/tsi_hold_ab.txt
done; done; unset FCG_LIB
bash tools/probes/r06.sh suite smoke bench || exit 1
