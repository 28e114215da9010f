#!/bin/bash
# Round-6 GPU probe runner.  usage (on the GPU box, from the repo root): tools/probes/r06.sh <step>...
# Every step runs under its own time limit; the first failing step ends the call.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r06
mkdir -p $O
export TMPDIR=/tmp
ET="tools/eval_timing.py"
PT="python3 -u -m pytest -x -v --timeout 170 --timeout-method thread"
run() {  # run <seconds> <log> <cmd...>: time-limited, output appended to $O/<log>
  local t=$1 log=$2; shift 2
  echo "== $*" >> $O/$log
  timeout -k 10 "$t" "$@" >> $O/$log 2>&1 || { echo "step failed ($?): $*"; tail -40 $O/$log; exit 1; }
}
for step in "$@"; do
  case $step in
    new)    # this round's new GPU tests
      run 600 new_tests.log $PT tests/test_multigpu.py tests/test_integration_cxx.py -m gpu \
        -k "async or failure or inject" ;;
    sel)    # PYTEST_SEL="<files/-k ...>"
      run 900 sel_tests.log $PT -m gpu $PYTEST_SEL ;;
    suite)  # the whole GPU suite
      run 1000 gpu_tests.log $PT tests -m gpu ;;
    smoke)
      run 300 smoke.log python3 -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)  # the driver's default bench
      run 900 bench.log python3 bench.py && grep '^{' $O/bench.log | tail -1 > $O/bench.json ;;
    benchp) # primary line only
      run 300 benchp.log python3 bench.py --only-primary && grep '^{' $O/benchp.log | tail -1 > $O/benchp.json ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "r06 steps done: $*"
