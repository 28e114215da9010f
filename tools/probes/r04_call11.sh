#!/bin/bash
# round 4, call 11: lattice-ordered sum-factorised apply -- tests, timing, kernel stats + counters
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r04
mkdir -p $O/apply_stats
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_tangent_apply.py \
  > $O/call11_tests.log 2>&1; rc=$?
tail -n 3 $O/call11_tests.log
[ $rc -eq 0 ] || exit $rc
for k in totlag linear; do
  timeout -k 10 300 python tools/probes/apply_timing.py --n 100 --kinem $k 2>&1 | tail -n 1 | tee -a $O/apply_timing_lat.jsonl || exit 1
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/apply_stats" -o run -- \
  python3 "$GRAFT_REPO_ROOT/tools/probes/apply_timing.py" --n 100 --kinem totlag --reps 10) > $O/apply_stats.log 2>&1 || exit 1
f=$(find $O/apply_stats -name "*kernel_stats.csv" | head -1); head -12 "$f"
PMC_SCRIPT=tools/probes/apply_timing.py timeout -k 10 600 bash tools/pmc_kernel.sh r04/apply_pmc apply_sf occ,inst,mem -- --n 60 --kinem totlag --reps 3 || exit 1
