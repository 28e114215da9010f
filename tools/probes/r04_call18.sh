#!/bin/bash
# round 4, call 18: wavefront-per-workgroup matrix-free apply -- tests, A/B timing (wave vs sf), Newton
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_tangent_apply.py \
  > $O/call18_tests.log 2>&1; rc=$?
tail -n 3 $O/call18_tests.log
[ $rc -eq 0 ] || exit $rc
for k in totlag linear; do
  for v in wave sf; do
    FCG_H27_APPLY=$v timeout -k 10 300 python tools/probes/apply_timing.py --n 100 --kinem $k 2>&1 | tail -n 1 | sed "s/^{/{\"kernel\": \"$v\", /" | tee -a $O/apply_timing_wave.jsonl || exit 1
  done
done
timeout -k 10 500 python tools/newton_bench.py --celltype hex27 --kinem totlag --n 100 --length 1 --load -1 --mg --mg-matrix-free \
  > $O/newton27_w.json 2> $O/newton27_w.err || exit 1
python -c "import json; d=json.loads(open('$O/newton27_w.json').read().strip().splitlines()[-1]); print({k: d[k] for k in ('newton_s','solve_ms_total','pcg_iterations','tip_uz')})"
