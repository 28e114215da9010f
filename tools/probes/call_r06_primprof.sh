#!/bin/bash
# rocprofv3 kernel statistics of the headline alone (bench.py --only-primary) on the final build
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=$GRAFT_REPO_ROOT/gpurun_out/r06; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/primprof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --only-primary > $O/primprof_bench.json 2> $O/primprof.err || { tail -20 $O/primprof.err; exit 1; }
head -4 $O/primprof/run_kernel_stats.csv
