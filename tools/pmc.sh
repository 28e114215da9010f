#!/bin/bash
# rocprofv3 counter passes (each pass its own run, no tracing domains mixed in).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
TAG=${1:-pmc}; shift
ARGS="$@"
export TMPDIR=/tmp
OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
         "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  (cd /tmp && timeout -k 10 240 rocprofv3 --pmc $C --output-format csv -d "$OUT/p$i" -o run -- python3 "$GRAFT_REPO_ROOT/${PMC_SCRIPT:-tools/prof_kernel.py}" $ARGS) > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/p$i.log"; exit $rc; fi
done
