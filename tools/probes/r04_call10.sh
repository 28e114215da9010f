#!/bin/bash
# round 4, call 10: sum-factorised matrix-free hex27 action -- parity tests, A/B timing vs the direct kernel, config-3 Newton
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 400 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_tangent_apply.py \
  > $O/call10_tests.log 2>&1; rc=$?
tail -n 12 $O/call10_tests.log
[ $rc -eq 0 ] || exit $rc
for cfg in "100 totlag" "100 linear"; do
  set -- $cfg
  for v in sf direct; do
    FCG_H27_APPLY=$v timeout -k 10 300 python tools/probes/apply_timing.py --n $1 --kinem $2 2>&1 | tail -n 1 | sed "s/^{/{\"kernel\": \"$v\", /" | tee -a $O/apply_timing_sf.jsonl || exit 1
  done
done
timeout -k 10 500 python tools/newton_bench.py --celltype hex27 --kinem totlag --n 100 --length 1 --load -1 --mg --mg-matrix-free \
  > $O/newton27_sf.json 2> $O/newton27_sf.err || exit 1
tail -c 600 $O/newton27_sf.json; echo
