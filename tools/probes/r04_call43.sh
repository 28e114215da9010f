#!/bin/bash
# round 4, call 43: kernel statistics of the two Newton lines at the final build
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r04
mkdir -p $O/final_amg $O/final_c3
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/final_amg" -o run -- \
  python3 "$GRAFT_REPO_ROOT/tools/newton_bench.py" --celltype hex8 --kinem totlag --n 100 --length 1 --load=-1e-2 --renumber --amg-native) > $O/final_amg.log 2>&1 || exit 1
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/final_c3" -o run -- \
  python3 "$GRAFT_REPO_ROOT/tools/newton_bench.py" --celltype hex27 --kinem totlag --n 100 --length 1 --load -1 --mg --mg-matrix-free --mg-outer-matrix-free) > $O/final_c3.log 2>&1 || exit 1
head -6 $O/final_amg/run_kernel_stats.csv | cut -c1-120
head -6 $O/final_c3/run_kernel_stats.csv | cut -c1-120
