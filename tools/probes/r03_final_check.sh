#!/bin/bash
# Round-3 final check at HEAD on one MI355X: smoke, the whole -m gpu suite, the default bench line,
# and the self-launched 2-rank rehearsal (gloo, both ranks on GPU 0).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
TAG=${TAG:-r03_final}
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/${TAG}_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 450 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${TAG}_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_bench.err; exit $rc; }
python3 -c "
import json; d=json.loads(open('gpurun_out/${TAG}_bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'ms_per_step', d['ms_per_step'], 'frac', d['roofline']['frac'])"
FCG_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline \
  > gpurun_out/${TAG}_bench_gloo2.json 2> gpurun_out/${TAG}_bench_gloo2.err
rc=$?; echo "bench gloo2 rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_bench_gloo2.err; exit $rc; }
python3 -c "
import json; d=json.loads(open('gpurun_out/${TAG}_bench_gloo2.json').read().strip().splitlines()[-1])
print('gloo2 n_gpus', d['n_gpus'], 'elements_global', d['config']['elements_global'], 'value', d['value'])"
