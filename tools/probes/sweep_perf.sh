set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_visit_table.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/sweep_tests.log 2>&1 || { tail -30 gpurun_out/sweep_tests.log; exit 1; }
tail -2 gpurun_out/sweep_tests.log
for k in linear totlag; do
  timeout -k 10 120 python tools/eval_timing.py --celltype hex8 --kinem $k --n 100 --path structured --reps 15 || exit 1
done
