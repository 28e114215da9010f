#!/bin/bash
# Round-3 profiles at HEAD on one MI355X: rocprofv3 kernel stats of the default bench (N=1) and
# HBM traffic (PMC, separate passes) of the hex27 element + row-assembly kernels at 40^3 TotLag.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
TAG=${TAG:-r03_final}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_bench_prof -o run -- \
  python3 bench.py --steps 20 --warmup 5 --no-newton --no-amg --no-cpu-baseline > gpurun_out/${TAG}_bench_prof.json 2> gpurun_out/${TAG}_bench_prof.err
rc=$?; echo "bench prof rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_bench_prof.err; exit $rc; }
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/${TAG}_h27_pmc/$C -o run -- \
    python3 tools/prof_kernel.py --celltype hex27 --kinem totlag --n 40 --reps 3 > gpurun_out/${TAG}_h27_pmc_$C.log 2>&1
  rc=$?; echo "h27 pmc $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
