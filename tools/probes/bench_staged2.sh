#!/bin/bash
# Rehearsal of bench.py's multi-rank flow on one GPU: 2 ranks over torch.distributed.run with the
# host-staged gloo transport (RCCL refuses two ranks on one device); the driver's N-GPU runs use RCCL.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
FCG_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline \
  > gpurun_out/bench_staged2.json 2> gpurun_out/bench_staged2.err
rc=$?; tail -c 1500 gpurun_out/bench_staged2.json; tail -3 gpurun_out/bench_staged2.err; exit $rc
