# hex27 pair phase: MFMA (default) vs the VALU loop (FCG_H27_MFMA=0): parity tests with MFMA on,
# then evaluate timings at 40^3 for both kinematics and both settings, general and coloured paths.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_tsi.py tests/test_newton_gpu.py -q -x -k "27 or hex27 or h27 or newton" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/h27_tests.log 2>&1 || { tail -30 gpurun_out/h27_tests.log; exit 1; }
tail -1 gpurun_out/h27_tests.log
for kin in linear totlag; do
for path in general structured; do
for mf in 1 0; do
FCG_H27_MFMA=$mf timeout -k 10 200 python tools/eval_timing.py --celltype hex27 --kinem $kin --n ${N:-40} --path $path > gpurun_out/h27_${kin}_${path}_${mf}.json 2> gpurun_out/h27.err || { tail -20 gpurun_out/h27.err; exit 1; }
echo "$kin $path mfma=$mf $(cat gpurun_out/h27_${kin}_${path}_${mf}.json | cut -c1-400)"
done; done; done
