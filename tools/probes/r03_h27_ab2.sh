#!/bin/bash
# hex27 A/B on one box: default build vs the FCG_LIB variants named in $VARIANTS (40^3 TotLag)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
TAG=${TAG:-r03_h27_ab2}
mkdir -p gpurun_out
for rep in 1 2; do
  for v in default ${VARIANTS}; do
    if [ "$v" = default ]; then unset FCG_LIB; else export FCG_LIB=$v; fi
    timeout -k 10 120 python tools/eval_timing.py --celltype hex27 --kinem ${KIN:-totlag} --n 40 --reps 7 --path general | sed "s/^/$v /" >> gpurun_out/${TAG}_timing.txt || exit 1
  done
done
unset FCG_LIB
python3 - gpurun_out/${TAG}_timing.txt <<'PY'
import json, sys
for line in open(sys.argv[1]):
    tag = line.split("{")[0].strip(); d = json.loads(line[line.index("{"):])
    print(f"{tag:12s} evaluate {d['ms_evaluate']:.3f} element {d['ms_element']:.3f} assemble {d['ms_assemble']:.3f}")
PY
