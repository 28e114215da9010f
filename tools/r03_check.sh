#!/bin/bash
# Round-3 check on one MI355X: the new GPU tests, the default bench line (N=1, in-run PMC
# traffic) and the self-launched 2-rank rehearsal (FCG_DIST_BACKEND=gloo, both ranks on GPU 0).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
TAG=${TAG:-r03_v1}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_missing_device.py tests/test_newton_gpu.py tests/test_multigpu.py \
  > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/${TAG}_bench.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_bench.err; exit $rc; }
FCG_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline \
  > gpurun_out/${TAG}_bench_gloo2.json 2> gpurun_out/${TAG}_bench_gloo2.err
rc=$?; echo "bench gloo2 rc=$rc"; tail -c 600 gpurun_out/${TAG}_bench_gloo2.json; [ $rc -eq 0 ] || tail -20 gpurun_out/${TAG}_bench_gloo2.err
exit $rc
