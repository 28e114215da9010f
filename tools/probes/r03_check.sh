#!/bin/bash
# Round-3 check on one MI355X: the new GPU tests, the default bench line (N=1, in-run PMC
# traffic) and the self-launched 2-rank rehearsal (FCG_DIST_BACKEND=gloo, both ranks on GPU 0).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
TAG=${TAG:-r03_v1}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_missing_device.py tests/test_newton_gpu.py tests/test_multigpu.py tests/test_gather_tiled.py \
  "tests/test_gpu_parity.py" \
  > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/${TAG}_bench.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_bench.err; exit $rc; }
FCG_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline \
  > gpurun_out/${TAG}_bench_gloo2.json 2> gpurun_out/${TAG}_bench_gloo2.err
rc=$?; echo "bench gloo2 rc=$rc"; tail -c 600 gpurun_out/${TAG}_bench_gloo2.json; [ $rc -eq 0 ] || tail -20 gpurun_out/${TAG}_bench_gloo2.err
[ $rc -eq 0 ] || exit $rc
for C in FETCH_SIZE WRITE_SIZE; do
  (cd /tmp && timeout -k 10 120 rocprofv3 --pmc $C --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_gather_pmc/$C" -o run -- \
    python3 "$GRAFT_REPO_ROOT/tools/prof_kernel.py" --renumber --reps 3) > gpurun_out/${TAG}_gather_pmc_$C.log 2>&1
  rc=$?; echo "gather pmc $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 500 python -u -m pytest -x -v --timeout 450 --timeout-method thread -p no:cacheprovider \
  tests/test_config3_fullsize.py "tests/test_fullsize.py::test_config3_newton_equilibrium_and_symmetry" \
  > gpurun_out/${TAG}_config3.log 2>&1
rc=$?; echo "config3 rc=$rc"; tail -4 gpurun_out/${TAG}_config3.log
exit $rc
