#!/bin/bash
# round 4, call 12: matrix-free apply (lattice layouts) + non-nested coarse levels -- tests, timing, config-3 Newton, kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r04
mkdir -p $O/newton_stats
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_tangent_apply.py tests/test_multigrid.py \
  > $O/call12_tests.log 2>&1; rc=$?
tail -n 3 $O/call12_tests.log
[ $rc -eq 0 ] || exit $rc
for k in totlag linear; do
  timeout -k 10 300 python tools/probes/apply_timing.py --n 100 --kinem $k 2>&1 | tail -n 1 | tee -a $O/apply_timing_lat.jsonl || exit 1
done
timeout -k 10 500 python tools/newton_bench.py --celltype hex27 --kinem totlag --n 100 --length 1 --load -1 --mg --mg-matrix-free \
  > $O/newton27_nn.json 2> $O/newton27_nn.err || exit 1
python -c "import json; d=json.loads(open('$O/newton27_nn.json').read().strip().splitlines()[-1]); print({k: d[k] for k in ('newton_s','solve_ms_total','pcg_iterations','mg_levels')})"
(cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/newton_stats" -o run -- \
  python3 "$GRAFT_REPO_ROOT/tools/newton_bench.py" --celltype hex27 --kinem totlag --n 100 --length 1 --load -1 --mg --mg-matrix-free) > $O/newton_stats.log 2>&1 || exit 1
f=$(find $O/newton_stats -name "*kernel_stats.csv" | head -1); head -16 "$f" | cut -c1-160
