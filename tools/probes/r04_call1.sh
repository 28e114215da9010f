#!/bin/bash
# round 4, first GPU call: counter list, the new config-4 / refusal tests, sweep counters at HEAD
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r04
mkdir -p $O
(cd /tmp && timeout -k 10 60 rocprofv3 -L) > $O/counters.txt 2>&1 || echo "rocprofv3 -L rc=$?"
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
  tests/test_config4_fullsize.py \
  tests/test_multigpu.py -k "config4 or refuses or native_dfcg" 2>&1 | tee $O/tests.log || exit 1
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
         "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC" \
         "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$GRAFT_REPO_ROOT/$O/sweep/p$i" -o run -- python3 "$GRAFT_REPO_ROOT/tools/prof_kernel.py" --n 100 --reps 3) > $O/sweep_p$i.log 2>&1
  echo "pass $i rc=$?"
done
python3 tools/pmc_summary.py $O/sweep "sweep_h8_kernel" > $O/sweep_pmc_summary.txt 2>&1
cat $O/sweep_pmc_summary.txt
