#!/bin/bash
# One GPU-box pass: gpu tests, then (if they ran without a fault) a short bench and a rocprofv3
# kernel-trace of the same bench.  Every GPU step has its own time limit; a crash/timeout stops
# the script (exit codes > 1 from pytest, non-zero from bench).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
TAG=${1:-r01}
timeout -k 10 700 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/gpu_tests_$TAG.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench_$TAG.json; tail -3 gpurun_out/bench_$TAG.err
if [ $rc -ne 0 ]; then exit $rc; fi
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --no-newton --no-amg > "$GRAFT_REPO_ROOT/gpurun_out/bench_prof_$TAG.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/bench_prof_$TAG.err"
rc=$?
echo "rocprof rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
# HBM traffic of the evaluate kernel (separate counter passes), for bench.py roofline.traffic
bash "$GRAFT_REPO_ROOT/tools/pmc.sh" "pmc_$TAG" --n 100 --reps 3
rc=$?
echo "pmc rc=$rc"
exit $rc
