#!/bin/bash
# hex27 matrix-core element kernel + symmetric-record assembly (fcg_hex27.hip): parity, then
# timing against the incidence-record kernels (FCG_H27_LEGACY=1), a rocprofv3 kernel trace and
# the counter passes of tools/pmc.sh for both kernels.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
TAG=${TAG:-r03_h27_v2}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py tests/test_newton_gpu.py "tests/test_fullsize.py::test_totlag_full_size_against_oracle" \
  > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
for K in linear totlag; do
  timeout -k 10 120 python tools/eval_timing.py --celltype hex27 --kinem $K --n 40 --reps 7 >> gpurun_out/${TAG}_timing.jsonl || exit 1
done
timeout -k 10 200 python tools/eval_timing.py --celltype hex27 --kinem totlag --n 100 --reps 5 >> gpurun_out/${TAG}_timing.jsonl || exit 1
cat gpurun_out/${TAG}_timing.jsonl
(cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof" -o run -- \
  python3 "$GRAFT_REPO_ROOT/tools/eval_timing.py" --celltype hex27 --kinem totlag --n 40 --reps 5) > gpurun_out/${TAG}_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
PMC_SCRIPT=tools/eval_timing.py bash tools/pmc.sh ${TAG}_pmc --celltype hex27 --kinem totlag --n 40 --reps 3 || exit 1
python3 tools/pmc_summary.py gpurun_out/${TAG}_pmc h27_element > gpurun_out/${TAG}_pmc_element.txt
python3 tools/pmc_summary.py gpurun_out/${TAG}_pmc h27_assemble > gpurun_out/${TAG}_pmc_assemble.txt
cat gpurun_out/${TAG}_pmc_element.txt gpurun_out/${TAG}_pmc_assemble.txt
timeout -k 10 500 python -u -m pytest -x -v --timeout 450 --timeout-method thread -p no:cacheprovider \
  tests/test_config3_fullsize.py > gpurun_out/${TAG}_config3.log 2>&1
rc=$?; echo "config3 rc=$rc"; tail -3 gpurun_out/${TAG}_config3.log
exit $rc
