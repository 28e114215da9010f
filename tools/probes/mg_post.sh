#!/bin/bash
# config 3 (1M hex27 StVK TotLag full Newton, geometric multigrid FCG): the default V-cycle against
# pre-smoothing only on the finest level (--mg-no-fine-post), Chebyshev degree 2 and 3
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
run() {
  timeout -k 10 300 python tools/newton_bench.py --celltype hex27 --kinem totlag --n 100 --length 1 --load -1 --mg "$@" > gpurun_out/mgp.json 2> gpurun_out/mgp.err || { tail -5 gpurun_out/mgp.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/mgp.json')); print(sys.argv[1:], round(d['newton_s'],3), d['pcg_iterations'], d.get('tip_uz'))" "$@"
}
run
run --mg-no-fine-post
run --mg-no-fine-post --mg-nu 3
run
