#!/bin/bash
# round 4, call 7: coupled AMG with the globally smoothed prolongator (2 / 4 / 8 ranks, native C++)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 900 python -u -m pytest -v -s --timeout 600 --timeout-method thread \
  tests/test_multigpu.py -k "native_dfcg or many_ranks or refuses" 2>&1 | tee $O/call7_tests.log | grep -E "PASS|FAIL|passed|failed|FCG iter|Error|assert" ; rc=${PIPESTATUS[0]}
timeout -k 10 400 tests/cxx/_build/config3_native 40 2 > $O/cxx_config3_native_40_v2.log 2>&1; rc2=$?
tail -3 $O/cxx_config3_native_40_v2.log
timeout -k 10 400 tests/cxx/_build/config3_native 16 4 > $O/cxx_config3_native_16x4.log 2>&1; rc3=$?
tail -3 $O/cxx_config3_native_16x4.log
exit $((rc | rc2 | rc3))
