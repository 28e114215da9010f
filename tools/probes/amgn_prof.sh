set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_amgn -o amgn -- python3 $GRAFT_REPO_ROOT/tools/newton_bench.py --celltype hex8 --kinem totlag --n 100 --length 1 --load=-1e-2 --renumber --amg-native > $GRAFT_REPO_ROOT/gpurun_out/amgn_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/amgn_prof.err || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/amgn_prof.err; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/prof_amgn -name "*kernel_stats.csv"
