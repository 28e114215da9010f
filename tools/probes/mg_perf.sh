set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_multigrid.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/mg_tests.log 2>&1 || { tail -30 gpurun_out/mg_tests.log; exit 1; }
tail -2 gpurun_out/mg_tests.log
timeout -k 10 400 python tools/newton_bench.py --celltype hex27 --kinem totlag --n 100 --length 1 --load -1 --mg --mg-mixed || exit 1
timeout -k 10 400 python tools/newton_bench.py --celltype hex27 --kinem totlag --n 100 --length 1 --load -1 --mg || exit 1
