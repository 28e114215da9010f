# config 3 (1M hex27 TotLag full Newton, geometric multigrid) with different Chebyshev eigenvalue ratios
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in ${RATIOS:-10 30}; do
timeout -k 10 400 python tools/newton_bench.py --celltype hex27 --kinem totlag --n 100 --length 1 --load=-1 --mg --mg-ratio $r > gpurun_out/mgr_$r.json 2> gpurun_out/mgr_$r.err || { tail -20 gpurun_out/mgr_$r.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/mgr_$r.json'))
print('ratio $r', round(d['newton_s'],3), d['pcg_iterations'], round(d['solve_ms_total'],1))"
done
