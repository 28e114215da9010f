# The Newton solvers after a change to the cycle: multigrid + AMG GPU tests, config 3 (1M hex27
# TotLag, geometric multigrid), and the 1M renumbered hex8 box with AMG (linear, TotLag).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_multigrid.py tests/test_amg.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/solver_tests.log 2>&1 || { tail -30 gpurun_out/solver_tests.log; exit 1; }
tail -1 gpurun_out/solver_tests.log
[ -n "$NO_CFG3" ] || timeout -k 10 400 python tools/newton_bench.py --celltype hex27 --kinem totlag --n 100 --length 1 --load=-1 --mg > gpurun_out/cfg3_mg.json 2> gpurun_out/cfg3_mg.err || { tail -20 gpurun_out/cfg3_mg.err; exit 1; }
for kin in linear totlag; do
timeout -k 10 400 python tools/newton_bench.py --celltype hex8 --kinem $kin --n 100 --length 1 --load=-1e-2 --renumber --amg > gpurun_out/amg_${kin}.json 2> gpurun_out/amg_${kin}.err || { tail -20 gpurun_out/amg_${kin}.err; exit 1; }
done
