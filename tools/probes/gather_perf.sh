set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "gather" -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gather_tests.log 2>&1 || { tail -30 gpurun_out/gather_tests.log; exit 1; }
tail -2 gpurun_out/gather_tests.log
for k in linear totlag; do
  for p in gather general structured; do
    timeout -k 10 120 python tools/eval_timing.py --celltype hex8 --kinem $k --n 100 --path $p --reps 7 || exit 1
  done
  for p in gather general; do
    timeout -k 10 180 python tools/eval_timing.py --celltype hex8 --kinem $k --n 100 --path $p --reps 7 --renumber || exit 1
  done
done
