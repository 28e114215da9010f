#!/bin/bash
# Round-6 call: hex27 row-assembly batch-size A/B, HEAD counter sets of the gather (renumbered 1M,
# both kinematics) and of the hex27 TotLag element + row assembly kernels after the LDS layouts
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r06; mkdir -p $O
bash tools/probes/r06.sh suite smoke || exit 1
LIBS="default a27nb3 a27nb4 a27pf" bash tools/probes/r06.sh h27ab || exit 1
bash tools/probes/r06.sh gpmc || exit 1
timeout -k 10 600 tools/pmc_kernel.sh r06/h27pmc h27_element_kernel occ,inst,flop,mem -- --n 40 --celltype hex27 --kinem totlag --reps 3 > $O/h27pmc.log 2>&1 || { tail -20 $O/h27pmc.log; exit 1; }
python3 tools/pmc_summary.py $O/h27pmc assemble27_kernel > $O/h27pmc/summary_assemble27.txt 2>&1
tail -30 $O/h27pmc/summary.txt
