#!/bin/bash
# lattice detection: the new and touched GPU tests, then the gather / AUTO bench secondary at 1M
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
TAG=${TAG:-r03_detect}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py tests/test_gather_tiled.py -k "gather or tiled or renumbered or lattice" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
for p in auto gather; do
  timeout -k 10 300 python tools/eval_timing.py --celltype hex8 --kinem linear --n 100 --path $p --renumber --reps 10 >> gpurun_out/${TAG}_timing.jsonl || exit 1
done
cat gpurun_out/${TAG}_timing.jsonl
