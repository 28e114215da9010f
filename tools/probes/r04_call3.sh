#!/bin/bash
# round 4, call 3: coupled-AMG and gather tests, gather timing, then the full GPU suite + smoke + bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 800 --timeout-method thread \
  tests/test_multigpu.py tests/test_integration_cxx.py tests/test_gpu_parity.py tests/test_gather_tiled.py \
  -k "native or refuses or gather or negative or singular" 2>&1 | tee $O/call3_tests.log | grep -E "PASS|FAIL|passed|failed|FCG iter|Error" ; rc=${PIPESTATUS[0]}
[ $rc -eq 0 ] || exit $rc
for k in linear totlag; do
  timeout -k 10 200 python tools/eval_timing.py --n 100 --kinem $k --renumber --path gather --reps 20 | tail -1 | tee -a $O/gather_timing.jsonl || exit 1
done
ROUNDS=3 timeout -k 10 600 bash tools/exp_ab.sh default nopipe 2>&1 | tee $O/ab_visit_pipe.txt || exit 1
timeout -k 10 1500 python -u -m pytest -x -v --timeout 800 --timeout-method thread -m gpu tests > $O/gpu_tests_v1.log 2>&1; rc=$?
tail -5 $O/gpu_tests_v1.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tee $O/smoke_v1.log || exit 1
timeout -k 10 600 python bench.py > $O/bench_v1.json 2> $O/bench_v1.err; rc=$?
tail -c 1500 $O/bench_v1.json
exit $rc
