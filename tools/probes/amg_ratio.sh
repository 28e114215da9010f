set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_multigrid.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/mg_tests.log 2>&1 || { tail -30 gpurun_out/mg_tests.log; exit 1; }
tail -1 gpurun_out/mg_tests.log
for r in 10 20; do
timeout -k 10 400 python tools/newton_bench.py --celltype hex8 --kinem totlag --n 100 --length 1 --load=-1e-2 --renumber --amg-native --mg-ratio $r > gpurun_out/amgr_$r.json 2> gpurun_out/amgr_$r.err || { tail -20 gpurun_out/amgr_$r.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/amgr_$r.json'))
print('amg ratio $r', round(d['newton_s'],3), d['pcg_iterations'], round(d['solve_ms_total'],1))"
done
