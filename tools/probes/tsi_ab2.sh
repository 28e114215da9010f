# same-box A/B of the fused TSI sweep: FCG_LIB=base (lib/libfourc_gpu_base.so) vs the default build
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do
for v in base default; do
if [ $v = base ]; then export FCG_LIB=base; else unset FCG_LIB; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 10 --no-newton --no-amg --no-hex27 --no-optionb --no-host --no-gather --no-cpu-baseline > gpurun_out/tsi_ab.json 2> gpurun_out/tsi_ab.err || { tail -20 gpurun_out/tsi_ab.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/tsi_ab.json'))
print('$v', 'primary kernel', round(d['roofline']['ms_element_kernel'],4), 'tsi', [round(s['ms_per_step'],4) for s in d.get('secondary', [])])"
done; done
