#!/bin/bash
# round 4, call 20: counters of the wavefront-per-workgroup matrix-free apply
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
PMC_SCRIPT=tools/probes/apply_timing.py timeout -k 10 600 bash tools/pmc_kernel.sh r04/apply_pmc4 apply_sf occ,inst,mem -- --n 60 --kinem totlag --reps 3 || exit 1
