#!/bin/bash
# round 4, call 8: native C++ 4-rank coupled AMG at 32^3, then the full GPU suite + smoke + bench at HEAD
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 400 tests/cxx/_build/config3_native 32 4 > $O/cxx_config3_native_32x4.log 2>&1; rc=$?
tail -n 3 $O/cxx_config3_native_32x4.log
timeout -k 10 1500 python -u -m pytest -v --timeout 800 --timeout-method thread -m gpu tests > $O/gpu_tests_v2.log 2>&1; rc2=$?
tail -n 5 $O/gpu_tests_v2.log
[ $rc2 -eq 0 ] || [ $rc2 -eq 1 ] || exit $rc2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tee $O/smoke_v2.log || exit 1
timeout -k 10 600 python bench.py > $O/bench_v2.json 2> $O/bench_v2.err; rc3=$?
tail -c 600 $O/bench_v2.json
exit $((rc | rc2 | rc3))
