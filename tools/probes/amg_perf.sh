# AMG on MI355X: the GPU tests, then the Newton loop on the 1M-element renumbered hex8 box (the
# unstructured bench mesh) with AMG, against block-Jacobi PCG and the box's geometric multigrid.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
N=${N:-100}
timeout -k 10 400 python -u -m pytest tests/test_amg.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/amg_tests.log 2>&1 || { tail -30 gpurun_out/amg_tests.log; exit 1; }
tail -2 gpurun_out/amg_tests.log
for kin in ${KINS:-linear}; do
timeout -k 10 500 python tools/newton_bench.py --celltype hex8 --kinem $kin --n $N --length 1 --load=${LOAD:--1e-2} --renumber --amg > gpurun_out/amg_${kin}.json 2> gpurun_out/amg_${kin}.err || { tail -20 gpurun_out/amg_${kin}.err; exit 1; }
timeout -k 10 500 python tools/newton_bench.py --celltype hex8 --kinem $kin --n $N --length 1 --load=${LOAD:--1e-2} --mg > gpurun_out/gmg_${kin}.json 2> gpurun_out/gmg_${kin}.err || { tail -20 gpurun_out/gmg_${kin}.err; exit 1; }
done
if [ -n "$PCG" ]; then
timeout -k 10 900 python tools/newton_bench.py --celltype hex8 --kinem linear --n $N --length 1 --load=${LOAD:--1e-2} --renumber > gpurun_out/pcg_linear.json 2> gpurun_out/pcg_linear.err || { tail -20 gpurun_out/pcg_linear.err; exit 1; }
fi
