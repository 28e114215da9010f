#!/bin/bash
# round 4, call 4: TSI visit-pipelining A/B, gather counters, native config-3 iteration log,
# rocprof kernel statistics of the primary bench line alone
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r04
mkdir -p $O
TSI=1 NOLIN=1 ROUNDS=2 timeout -k 10 600 bash tools/exp_ab.sh default tsipipe 2>&1 | grep -v amdgpu.ids | tee $O/ab_tsi_pipe.txt || exit 1
for rep in 1 2; do for v in default gwpc8; do
  if [ "$v" = default ]; then unset FCG_LIB; else export FCG_LIB=$v; fi
  r=$(timeout -k 10 200 python tools/eval_timing.py --n 100 --renumber --path gather --reps 30 | tail -1) || exit 1
  echo "$v gather_linear $(echo "$r" | python3 -c 'import json,sys; print(round(json.load(sys.stdin)["ms_evaluate"],4))')" | tee -a $O/ab_gather_wpc.txt
done; done
unset FCG_LIB
timeout -k 10 400 tests/cxx/_build/config3_native 40 2 > $O/cxx_config3_native_40.log 2>&1 || exit 1
tail -4 $O/cxx_config3_native_40.log
bash tools/pmc_kernel.sh r04/gather "gather_h8_kernel<0, true, true, false>" occ,inst,flop,mem -- --n 100 --path gather --renumber --reps 3 > $O/gather_pmc.log 2>&1 || exit 1
tail -12 $O/gather/summary.txt
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prim" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --only-primary --steps 20 --warmup 5) > $O/prim_bench.json 2> $O/prim_bench.err || exit 1
tail -c 600 $O/prim_bench.json
find $O/prim -name "*kernel_stats.csv" | head -3
