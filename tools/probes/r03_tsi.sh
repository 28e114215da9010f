#!/bin/bash
# TSI two-field tangent: structural sweep + thermal-only pass (default) against the one fused
# pass (FCG_TSI_SPLIT=0): parity tests, timing at 126^3 (config 5), counters of the thermal pass.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
TAG=${TAG:-r03_tsi_v1}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_tsi.py > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tsi tests rc=$rc"; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
for S in 1 0; do
  FCG_TSI_SPLIT=$S timeout -k 10 200 python tools/tsi_bench.py --n 126 --reps 10 > gpurun_out/${TAG}_bench_split$S.json 2> gpurun_out/${TAG}_bench_split$S.err || exit 1
  tail -c 800 gpurun_out/${TAG}_bench_split$S.json
done
(cd /tmp && timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof" -o run -- \
  python3 "$GRAFT_REPO_ROOT/tools/tsi_bench.py" --n 126 --reps 5) > gpurun_out/${TAG}_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
for C in FETCH_SIZE WRITE_SIZE; do
  (cd /tmp && timeout -k 10 150 rocprofv3 --pmc $C --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_pmc/$C" -o run -- \
    python3 "$GRAFT_REPO_ROOT/tools/tsi_bench.py" --n 126 --reps 3) > gpurun_out/${TAG}_pmc_$C.log 2>&1
  rc=$?; echo "pmc $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
