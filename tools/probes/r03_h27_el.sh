#!/bin/bash
# hex27 element kernel: parity subset, general-path timing (40^3 TotLag / linear), phase stamps.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
TAG=${TAG:-r03_h27_el_v1}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py -k "27 or colored or singular or negative" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
for k in totlag linear; do
  timeout -k 10 150 python tools/eval_timing.py --celltype hex27 --kinem $k --n 40 --reps 7 --path general >> gpurun_out/${TAG}_timing.jsonl || exit 1
done
cat gpurun_out/${TAG}_timing.jsonl
timeout -k 10 200 python tools/h27_stamps.py 40 > gpurun_out/${TAG}_stamps.txt 2>&1 || exit 1
cat gpurun_out/${TAG}_stamps.txt
