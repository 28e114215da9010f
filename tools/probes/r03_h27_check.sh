#!/bin/bash
# hex27 at HEAD: parity tests (general path, config-3 rows straddling 2^31) and 40^3 / 100^3 timing
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
TAG=${TAG:-r03_h27_check}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 450 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py tests/test_config3_fullsize.py "tests/test_fullsize.py" -k "HEX27 or hex27 or 27 or config3" \
  > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
for n in 40 100; do
  timeout -k 10 300 python tools/eval_timing.py --celltype hex27 --kinem totlag --n $n --reps 5 --path general >> gpurun_out/${TAG}_timing.jsonl || exit 1
done
cat gpurun_out/${TAG}_timing.jsonl
