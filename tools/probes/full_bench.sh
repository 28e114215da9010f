cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { tail -20 gpurun_out/bench_full.err; exit 1; }
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r02 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-newton --no-amg --no-hex27 --no-cpu-baseline --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/bench_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/bench_prof.err || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/bench_prof.err; exit 1; }
ls $GRAFT_REPO_ROOT/gpurun_out/prof_r02
