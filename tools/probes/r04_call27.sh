#!/bin/bash
# round 4, call 27: matrix-free apply on odd element counts and a 125-element box (all three kernel variants)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r04
mkdir -p $O
for v in wave sf direct; do
  FCG_H27_APPLY=$v timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_tangent_apply.py -k "box_matches or renumbered" \
    > $O/call27_$v.log 2>&1 || { tail -n 20 $O/call27_$v.log; exit 1; }
  echo "$v: $(tail -n 1 $O/call27_$v.log)"
done
