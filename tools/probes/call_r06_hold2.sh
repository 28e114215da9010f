#!/bin/bash
# aligned hold buffers: the product build (linear hold rows 10 apart) against hold9 (round 5), the
# TotLag sweep with aligned rows (holdtl) and the deferred lower-plane buffer (holdlo10, renumbered
# mesh through AUTO), with the structured / deferred parity tests for each variant
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/r06
PYTEST_SEL="tests/test_gpu_parity.py tests/test_visit_table.py" bash tools/probes/r06.sh sel || exit 1
FCG_LIB=holdtl PYTEST_SEL="tests/test_gpu_parity.py tests/test_fullsize.py" bash tools/probes/r06.sh sel || exit 1
FCG_LIB=holdlo10 PYTEST_SEL="tests/test_gpu_parity.py" bash tools/probes/r06.sh sel || exit 1
LIBS="default hold9" ABTAG=linear ETARGS="--n 100 --reps 60" bash tools/probes/r06.sh libab || exit 1
LIBS="default holdtl" ABTAG=totlag ETARGS="--n 100 --kinem totlag --reps 30" bash tools/probes/r06.sh libab || exit 1
LIBS="default holdlo10" ABTAG=renum_auto ETARGS="--n 100 --renumber --reps 40" bash tools/probes/r06.sh libab || exit 1
LIBS="default hold9" ABTAG=linear ETARGS="--n 100 --reps 60" bash tools/probes/r06.sh libab || exit 1
