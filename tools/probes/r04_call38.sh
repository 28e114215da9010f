#!/bin/bash
# round 4, call 38: full GPU suite + smoke + default bench at HEAD (v6)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 1500 python -u -m pytest -v --timeout 800 --timeout-method thread -m gpu tests > $O/gpu_tests_v6.log 2>&1; rc=$?
tail -n 5 $O/gpu_tests_v6.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tee $O/smoke_v6.log || exit 1
timeout -k 10 900 python bench.py > $O/bench_v6.json 2> $O/bench_v6.err; rc3=$?
tail -c 400 $O/bench_v6.json
exit $((rc | rc3))
