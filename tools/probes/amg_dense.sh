#!/bin/bash
# native AMG: its GPU tests, then the renumbered 1M hex8 TotLag Newton with the dense coarsest
# inverse (default) and with the coarsest block-Jacobi CG (FCG_AMG_COARSE_CG=1), alternated
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_amg.py tests/test_integration_cxx.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/amgd_tests.log 2>&1 || { tail -30 gpurun_out/amgd_tests.log; exit 1; }
tail -1 gpurun_out/amgd_tests.log
for rep in 1 2; do
  for v in dense cg; do
    if [ $v = cg ]; then export FCG_AMG_COARSE_CG=1; else unset FCG_AMG_COARSE_CG; fi
    timeout -k 10 300 python tools/newton_bench.py --celltype hex8 --kinem totlag --n 100 --length 1 --load=-1e-2 --renumber --amg-native > gpurun_out/amgd_$v.json 2> gpurun_out/amgd_$v.err || { tail -20 gpurun_out/amgd_$v.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/amgd_$v.json')); print('$v', round(d['newton_s'],4), d['pcg_iterations'], [round(x,1) for x in d['amg_numeric_setup_ms']], d['tip_uz'])"
  done
done
