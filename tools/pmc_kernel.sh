#!/bin/bash
# rocprofv3 counter passes of one workload (each pass its own run, no tracing domains mixed in),
# summarised for the kernels whose name contains PATTERN.
#   tools/pmc_kernel.sh TAG PATTERN [SETS] -- <args of tools/prof_kernel.py>
# (PMC_SCRIPT=<repo-relative .py> profiles another workload script with those arguments)
# SETS (comma list): occ (wave / issue cycles), inst (instruction mix, LDS), flop (FP64 VALU and
# MFMA counts, matrix-pipe busy), mem (FETCH_SIZE, WRITE_SIZE, GRBM)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
TAG=$1; PAT=$2; SETS=${3:-occ,inst,flop,mem}; shift 3
[ "$1" == "--" ] && shift
export TMPDIR=/tmp
OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
declare -a P
[[ $SETS == *occ* ]] && P+=("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS")
[[ $SETS == *inst* ]] && P+=("SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE")
[[ $SETS == *flop* ]] && P+=("SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES")
[[ $SETS == *mem* ]] && P+=("FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT")
i=0
for C in "${P[@]}"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/p$i" -o run -- python3 "$GRAFT_REPO_ROOT/${PMC_SCRIPT:-tools/prof_kernel.py}" "$@") > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/p$i.log"; exit $rc; fi
done
python3 "$GRAFT_REPO_ROOT/tools/pmc_summary.py" "$OUT" "$PAT" > "$OUT/summary.txt" 2>&1
cat "$OUT/summary.txt"
