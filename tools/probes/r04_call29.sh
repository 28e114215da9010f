#!/bin/bash
# round 4, call 29: the multi-rank / C++-host tests with the dense coarsest inverse in the native AMG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_multigpu.py tests/test_integration_cxx.py tests/test_amg.py > $O/call29_tests.log 2>&1 || { tail -30 $O/call29_tests.log; exit 1; }
tail -3 $O/call29_tests.log
