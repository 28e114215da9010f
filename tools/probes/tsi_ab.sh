# TSI fused sweep A/B helper: parity tests of the fused path, then the config-5 timing
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_tsi.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tsi_tests.log 2>&1 || { tail -30 gpurun_out/tsi_tests.log; exit 1; }
tail -1 gpurun_out/tsi_tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 10 --no-newton --no-amg --no-hex27 --no-optionb --no-host --no-gather --no-cpu-baseline > gpurun_out/tsi_ab.json 2> gpurun_out/tsi_ab.err || { tail -20 gpurun_out/tsi_ab.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/tsi_ab.json'))
print('primary ms', d['ms_per_step'], 'kernel', d['roofline']['ms_element_kernel'])
for s in d.get('secondary', []): print(s['workload'], s.get('ms_per_step'))"
