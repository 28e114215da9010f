#!/bin/bash
# TSI split passes on two streams vs one after the other (FCG_TSI_CONCURRENT=0), same box; TSI tests
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
TAG=${TAG:-r03_tsi_conc}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 450 --timeout-method thread -p no:cacheprovider -m gpu tests/test_tsi.py > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tsi tests rc=$rc"; tail -1 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for c in 1 0; do
    FCG_TSI_CONCURRENT=$c timeout -k 10 200 python tools/tsi_bench.py --n 126 --reps 10 > gpurun_out/${TAG}_${c}_${rep}.json 2> gpurun_out/${TAG}.err || { tail -5 gpurun_out/${TAG}.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/${TAG}_${c}_${rep}.json').read().strip().splitlines()[-1])
print('concurrent=$c', {k: v for k, v in d.items() if 'ms' in k})"
  done
done
