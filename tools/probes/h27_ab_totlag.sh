set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do
for mf in 1 0; do
FCG_H27_MFMA=$mf timeout -k 10 200 python tools/eval_timing.py --celltype hex27 --kinem totlag --n 40 --path general > gpurun_out/h27_ab.json 2> gpurun_out/h27.err || { tail -20 gpurun_out/h27.err; exit 1; }
echo "totlag general mfma=$mf $(cut -c1-330 gpurun_out/h27_ab.json)"
done; done
