#!/bin/bash
# Row-block sweep on the 1M hex8 box, native numbering vs the renumbered (input-file) mesh that
# AUTO sends to the sweep by lattice detection: counter passes of tools/pmc.sh for the sweep kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
TAG=${TAG:-r03_renum}
mkdir -p gpurun_out
bash tools/pmc.sh ${TAG}_native --n 100 --reps 3 || exit 1
bash tools/pmc.sh ${TAG}_renum --n 100 --reps 3 --renumber || exit 1
python3 tools/pmc_summary.py gpurun_out/${TAG}_native sweep_h8 > gpurun_out/${TAG}_native_summary.txt
python3 tools/pmc_summary.py gpurun_out/${TAG}_renum sweep_h8 > gpurun_out/${TAG}_renum_summary.txt
paste gpurun_out/${TAG}_native_summary.txt gpurun_out/${TAG}_renum_summary.txt | cut -c1-150
