#!/bin/bash
# round 4, call 42: AMG / multi-rank / multigrid tests at the final build
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_amg.py tests/test_multigpu.py tests/test_multigrid.py > $O/call42_tests.log 2>&1 || { tail -30 $O/call42_tests.log; exit 1; }
tail -2 $O/call42_tests.log
