# gather path: parity tests, then 1M renumbered hex8 evaluate timings (linear, TotLag)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gather_tiled.py tests/test_gpu_parity.py -q -x -k "gather or tiled" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gather_tests.log 2>&1 || { tail -30 gpurun_out/gather_tests.log; exit 1; }
tail -1 gpurun_out/gather_tests.log
for kin in linear totlag; do
timeout -k 10 300 python tools/eval_timing.py --celltype hex8 --kinem $kin --n 100 --path gather --renumber --reps 10 > gpurun_out/gab_$kin.json 2> gpurun_out/gab.err || { tail -20 gpurun_out/gab.err; exit 1; }
echo "$kin $(cut -c1-300 gpurun_out/gab_$kin.json)"
done
