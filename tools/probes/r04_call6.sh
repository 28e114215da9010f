#!/bin/bash
# round 4, call 6: config 5 at full size against the oracle (1 and 8 ranks), coupled AMG at 4 / 8 ranks
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread \
  tests/test_tsi.py tests/test_multigpu.py -k "config5 or many_ranks" 2>&1 | tee $O/call6_tests.log | grep -E "PASS|FAIL|passed|failed|FCG iter|Error|assert" ; exit ${PIPESTATUS[0]}
