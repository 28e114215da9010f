#!/bin/bash
# Round-3 HEAD check on one MI355X: the whole -m gpu suite, the default bench line, hex27 timing.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
TAG=${TAG:-r03_head}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 450 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/${TAG}_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; tail -c 400 gpurun_out/${TAG}_bench.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_bench.err; exit $rc; }
for k in totlag linear; do
  timeout -k 10 120 python tools/eval_timing.py --celltype hex27 --kinem $k --n 40 --reps 7 >> gpurun_out/${TAG}_h27_timing.jsonl || exit 1
done
timeout -k 10 200 python tools/eval_timing.py --celltype hex27 --kinem totlag --n 100 --reps 5 >> gpurun_out/${TAG}_h27_timing.jsonl || exit 1
cat gpurun_out/${TAG}_h27_timing.jsonl
