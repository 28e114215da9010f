#!/bin/bash
# headline sweep: aligned hold buffer (FCG_HOLD10) against the product build, same box, 3 rounds,
# and the structured-path parity tests with it
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/r06
FCG_LIB=hold10 PYTEST_SEL="tests/test_gpu_parity.py tests/test_visit_table.py" bash tools/probes/r06.sh sel || exit 1
for i in 1 2 3; do
LIBS="default hold10" ABTAG=linear ETARGS="--n 100 --reps 60" bash tools/probes/r06.sh libab || exit 1
done
