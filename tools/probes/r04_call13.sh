#!/bin/bash
# round 4, call 13: XCD-contiguous persistent matrix-free apply -- tests, grid A/B, counters
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r04
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_tangent_apply.py \
  > $O/call13_tests.log 2>&1; rc=$?
tail -n 3 $O/call13_tests.log
[ $rc -eq 0 ] || exit $rc
for g in 512 1024 2048; do
  FCG_H27_APPLY_GRID=$g timeout -k 10 300 python tools/probes/apply_timing.py --n 100 --kinem totlag 2>&1 | tail -n 1 | sed "s/^{/{\"grid\": $g, /" | tee -a $O/apply_timing_xcd.jsonl || exit 1
done
timeout -k 10 300 python tools/probes/apply_timing.py --n 100 --kinem linear 2>&1 | tail -n 1 | tee -a $O/apply_timing_xcd.jsonl || exit 1
PMC_SCRIPT=tools/probes/apply_timing.py timeout -k 10 600 bash tools/pmc_kernel.sh r04/apply_pmc2 apply_sf occ,inst,mem -- --n 60 --kinem totlag --reps 3 || exit 1
