#!/bin/bash
# Round-6 end-of-session call: gather parity + the C-row shift A/B, the driver's default bench,
# and rocprofv3 kernel statistics of a bench run with the secondary lines (hex27, gather, TSI)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r06; mkdir -p $O
PYTEST_SEL="tests/test_gather_tiled.py tests/test_gpu_parity.py" bash tools/probes/r06.sh sel || exit 1
LIBS="default gc0" ABTAG=totlag ETARGS="--n 100 --renumber --path gather --kinem totlag --reps 30" bash tools/probes/r06.sh libab || exit 1
bash tools/probes/r06.sh bench || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-newton --no-slab --no-host --no-pmc --no-optionb --no-cpu-baseline --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$O/bench_prof.json 2> $GRAFT_REPO_ROOT/$O/bench_prof.err || { tail -20 $GRAFT_REPO_ROOT/$O/bench_prof.err; exit 1; }
find $GRAFT_REPO_ROOT/$O/prof -name "*kernel_stats.csv" | head
