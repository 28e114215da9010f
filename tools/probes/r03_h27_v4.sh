#!/bin/bash
# hex27 v4: incidence-record output (default) vs symmetric records (FCG_H27_SYMREC=1) vs the legacy
# kernels, 40^3 TotLag and linear, then 1M TotLag; hex27 parity subset first.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
TAG=${TAG:-r03_h27_v4}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py -k "27 or singular or negative or reproduc" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in ${VARIANTS:-default symrec legacy}; do
    case $v in
      default) unset FCG_H27_SYMREC; unset FCG_H27_LEGACY;;
      symrec) export FCG_H27_SYMREC=1; unset FCG_H27_LEGACY;;
      legacy) unset FCG_H27_SYMREC; export FCG_H27_LEGACY=1;;
      lin3) unset FCG_H27_SYMREC FCG_H27_LEGACY; export FCG_LIB=h27lin3;;
    esac
    [ "$v" = lin3 ] || unset FCG_LIB
    for k in totlag linear; do
      timeout -k 10 120 python tools/eval_timing.py --celltype hex27 --kinem $k --n 40 --reps 7 | sed "s/^/$v $k /" >> gpurun_out/${TAG}_timing.txt || exit 1
    done
  done
done
unset FCG_H27_SYMREC FCG_H27_LEGACY FCG_LIB
timeout -k 10 200 python tools/eval_timing.py --celltype hex27 --kinem totlag --n 100 --reps 5 | sed "s/^/1M /" >> gpurun_out/${TAG}_timing.txt || exit 1
timeout -k 10 200 python tools/h27_stamps.py 40 > gpurun_out/${TAG}_stamps.txt 2>&1 || exit 1
cat gpurun_out/${TAG}_stamps.txt
python3 - gpurun_out/${TAG}_timing.txt <<'PY'
import json, sys
for line in open(sys.argv[1]):
    tag = line.split("{")[0].strip(); d = json.loads(line[line.index("{"):])
    print(f"{tag:24s} evaluate {d['ms_evaluate']:.3f} element {d['ms_element']:.3f} assemble {d['ms_assemble']:.3f}")
PY
