#!/bin/bash
# round 4, call 26: where the native AMG Newton (renumbered 1M hex8 TotLag) spends its time
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r04
mkdir -p $O/amg_stats
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/amg_stats" -o run -- \
  python3 "$GRAFT_REPO_ROOT/tools/newton_bench.py" --celltype hex8 --kinem totlag --n 100 --length 1 --load=-1e-2 --renumber --amg-native) > $O/amg_stats.log 2>&1 || exit 1
tail -c 300 $O/amg_stats.log
