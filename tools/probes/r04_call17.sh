#!/bin/bash
# round 4, call 17: first-solve overheads of the graph FCG (capture, lambda_max estimate)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r04
mkdir -p $O
FCG_MG_GRAPH_TIMING=1 timeout -k 10 500 python tools/newton_bench.py --celltype hex27 --kinem totlag --n 100 --length 1 --load -1 --mg --mg-matrix-free \
  > $O/newton27_t.json 2> $O/newton27_t.err || exit 1
grep -E "captured|lambda_max|solve_ms" $O/newton27_t.err | cut -c1-200
