#!/bin/bash
# same-box timing of the TSI split pass: default build vs the FCG_LIB probe builds in $VARIANTS
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
TAG=${TAG:-r03_tsi_probe}
mkdir -p gpurun_out
for rep in 1 2; do
  for v in default ${VARIANTS}; do
    if [ "$v" = default ]; then unset FCG_LIB; else export FCG_LIB=$v; fi
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_${v}_${rep} -o run -- python3 tools/tsi_bench.py --n 126 --reps 5 > gpurun_out/${TAG}_${v}_${rep}.json 2> gpurun_out/${TAG}.err || { tail -5 gpurun_out/${TAG}.err; exit 1; }
    python3 - "$v" gpurun_out/${TAG}_${v}_${rep} <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[2] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "sweep_h8" in r["Name"]:
        print(sys.argv[1], r["Name"].split("<")[1].split(">")[0], r["Calls"], round(float(r["AverageNs"]) / 1e6, 3), "ms")
PY
  done
done
