#!/bin/bash
# hex27 TotLag: incidence records (default) vs one symmetric record per element (FCG_H27_SYMREC=1),
# 40^3 and 100^3 on one box
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
TAG=${TAG:-r03_symrec}
mkdir -p gpurun_out
for n in 40 100; do
  for s in 0 1; do
    FCG_H27_SYMREC=$s timeout -k 10 300 python tools/eval_timing.py --celltype hex27 --kinem totlag --n $n --reps 5 --path general \
      | sed "s/^/symrec=$s n=$n /" >> gpurun_out/${TAG}_timing.txt || exit 1
  done
done
cat gpurun_out/${TAG}_timing.txt
