cd $GRAFT_REPO_ROOT
for i in 1 2; do
for opt in "" "--timing-after"; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-newton --no-amg --no-hex27 --no-tsi --no-optionb --no-host --no-gather --no-cpu-baseline $opt > gpurun_out/bw.json 2>/dev/null || exit 1
python3 -c "
import json; d=json.loads(open('gpurun_out/bw.json').read().strip().split(chr(10))[-1]); print('$opt', round(d['ms_per_step'],4), round(d['roofline']['ms_element_kernel'],4))"
done; done
