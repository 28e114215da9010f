#!/bin/bash
# hex27 A/B: phase stamps, assembly grid sizes (FCG_H27_ASM_GRID), legacy kernels, 1M timing.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
TAG=${TAG:-r03_h27_v3}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py -k "27 or singular or negative or reproduc" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/h27_stamps.py 40 > gpurun_out/${TAG}_stamps.txt 2>&1 || exit 1
cat gpurun_out/${TAG}_stamps.txt
for G in 2048 4096 8192 16384; do
  FCG_H27_ASM_GRID=$G timeout -k 10 120 python tools/eval_timing.py --celltype hex27 --kinem totlag --n 40 --reps 7 | sed "s/^/grid=$G /" >> gpurun_out/${TAG}_timing.txt || exit 1
done
FCG_H27_HVALU=1 timeout -k 10 120 python tools/eval_timing.py --celltype hex27 --kinem totlag --n 40 --reps 7 | sed "s/^/hvalu /" >> gpurun_out/${TAG}_timing.txt || exit 1
FCG_H27_HVALU=1 timeout -k 10 200 python tools/h27_stamps.py 40 > gpurun_out/${TAG}_stamps_hvalu.txt 2>&1 || exit 1
FCG_H27_LEGACY=1 timeout -k 10 120 python tools/eval_timing.py --celltype hex27 --kinem totlag --n 40 --reps 7 | sed "s/^/legacy /" >> gpurun_out/${TAG}_timing.txt || exit 1
timeout -k 10 200 python tools/eval_timing.py --celltype hex27 --kinem totlag --n 100 --reps 5 | sed "s/^/1M /" >> gpurun_out/${TAG}_timing.txt || exit 1
cat gpurun_out/${TAG}_timing.txt
