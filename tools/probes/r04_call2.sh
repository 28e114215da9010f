#!/bin/bash
# round 4, call 2: refusal test; HEAD counter sets of the three kernels VERDICT r3 names
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_multigpu.py -k "refuses" 2>&1 | tee $O/tests2.log || exit 1
bash tools/pmc_kernel.sh r04/sweep "sweep_h8_kernel<0, true, true, 0>" occ,inst,flop,mem -- --n 100 --reps 3 || exit 1
bash tools/pmc_kernel.sh r04/h27 "h27_element" occ,inst,flop,mem -- --n 40 --celltype hex27 --kinem totlag --reps 3 || exit 1
bash tools/pmc_kernel.sh r04/tsi_th "true, 2>" occ,inst,flop,mem -- --n 126 --tsi --reps 3 || exit 1
