# rocprofv3 kernel stats of the AMG Newton loop on the renumbered 1M hex8 box (and of the box's
# geometric multigrid for comparison)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
N=${N:-100}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_amg -o amg -- python3 tools/newton_bench.py --celltype hex8 --kinem linear --n $N --length 1 --load=-1e-2 --renumber --amg > gpurun_out/amg_prof.json 2> gpurun_out/amg_prof.err || { tail -20 gpurun_out/amg_prof.err; exit 1; }
find gpurun_out/prof_amg -name "*kernel_stats.csv" | head -3
