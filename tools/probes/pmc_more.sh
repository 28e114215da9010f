# PMC passes (tools/pmc.sh) of the hex27 TotLag general path (40^3) and of the gather path on the
# renumbered 1M hex8 box (linear, TotLag)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/pmc.sh pmc_h27 --celltype hex27 --kinem totlag --n 40 --path general --reps 3 || exit 1
bash tools/pmc.sh pmc_gl --n 100 --path gather --renumber --reps 3 || exit 1
bash tools/pmc.sh pmc_gt --n 100 --kinem totlag --path gather --renumber --reps 3 || exit 1
