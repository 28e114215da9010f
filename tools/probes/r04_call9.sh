#!/bin/bash
# round 4, call 9: matrix-free hex27 tangent action -- parity tests, operator timing, config-3 Newton A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 400 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_tangent_apply.py \
  > $O/call9_tests.log 2>&1; rc=$?
tail -n 15 $O/call9_tests.log
[ $rc -eq 0 ] || exit $rc
for cfg in "40 totlag" "100 totlag" "100 linear"; do
  set -- $cfg
  timeout -k 10 300 python tools/probes/apply_timing.py --n $1 --kinem $2 2>&1 | tail -n 1 | tee -a $O/apply_timing.jsonl || exit 1
done
for mf in "" "--mg-matrix-free"; do
  timeout -k 10 500 python tools/newton_bench.py --celltype hex27 --kinem totlag --n 100 --length 1 --load -1 --mg $mf \
    > $O/newton27_mf$([ -n "$mf" ] && echo 1 || echo 0).json 2> $O/newton27_mf$([ -n "$mf" ] && echo 1 || echo 0).err || exit 1
  tail -c 900 $O/newton27_mf$([ -n "$mf" ] && echo 1 || echo 0).json; echo
done
