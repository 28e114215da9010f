#!/bin/bash
# round 4, call 32: where config 3's Newton goes now (kernel stats, matrix-free outer + fused
# Chebyshev)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r04
mkdir -p $O/c3_stats
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/c3_stats" -o run -- \
  python3 "$GRAFT_REPO_ROOT/tools/newton_bench.py" --celltype hex27 --kinem totlag --n 100 --length 1 --load -1 --mg --mg-matrix-free --mg-outer-matrix-free) > $O/c3_stats.log 2>&1 || exit 1
python3 - <<'PY'
import csv
r=list(csv.DictReader(open('gpurun_out/r04/c3_stats/run_kernel_stats.csv')))
tot=sum(float(x['TotalDurationNs']) for x in r)
for x in r[:30]:
    print(x['Name'][:80], x['Calls'], round(float(x['TotalDurationNs'])/1e6,2), round(float(x['AverageNs'])/1e3,1))
print('total ms', tot/1e6)
PY
grep -o '"newton_s": [0-9.]*' $O/c3_stats.log
