#!/bin/bash
# Native distributed solve (fcg_dfcg_solve): 2-rank host-staged tests and the C++ host solving
# config 3 natively.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
TAG=${TAG:-r03_ds_v1}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  "tests/test_multigpu.py::test_two_ranks_native_dfcg" tests/test_integration_cxx.py tests/test_amg.py \
  > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "dsolve tests rc=$rc"; grep -E "PASS|FAIL|passed|failed|Error" gpurun_out/${TAG}_tests.log | tail -15
exit $rc
