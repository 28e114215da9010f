#!/bin/bash
# round 4, call 24: TSI thermal pass with / without its plane prefetch (timing probe)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r04
mkdir -p $O
TSI=1 NOLIN=1 ROUNDS=2 timeout -k 10 900 bash tools/exp_ab.sh default thnostore th1store 2>&1 | grep -v amdgpu.ids | tee $O/ab_th_stores.txt || exit 1
