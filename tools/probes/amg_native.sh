# Native (C-ABI) AMG: its GPU tests, then the 1M renumbered hex8 Newton with it (linear, TotLag).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_amg.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/amgn_tests.log 2>&1 || { tail -40 gpurun_out/amgn_tests.log; exit 1; }
tail -1 gpurun_out/amgn_tests.log
for kin in linear totlag; do
timeout -k 10 400 python tools/newton_bench.py --celltype hex8 --kinem $kin --n ${N:-100} --length 1 --load=-1e-2 --renumber --amg-native > gpurun_out/amgn_${kin}.json 2> gpurun_out/amgn_${kin}.err || { tail -20 gpurun_out/amgn_${kin}.err; exit 1; }
done
