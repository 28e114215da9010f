# config 3 with the geometric multigrid's coarsest level solved by block-Jacobi PCG vs the native AMG
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_multigrid.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/mg_tests.log 2>&1 || { tail -30 gpurun_out/mg_tests.log; exit 1; }
tail -1 gpurun_out/mg_tests.log
for c in amg pcg; do
timeout -k 10 400 python tools/newton_bench.py --celltype hex27 --kinem totlag --n 100 --length 1 --load=-1 --mg --mg-coarse $c > gpurun_out/mgc_$c.json 2> gpurun_out/mgc_$c.err || { tail -20 gpurun_out/mgc_$c.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/mgc_$c.json'))
print('coarse $c', round(d['newton_s'],3), d['pcg_iterations'], round(d['solve_ms_total'],1), round(d['setup_s'],1), d['tip_uz'])"
done
