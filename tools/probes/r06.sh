#!/bin/bash
# Round-6 GPU probe runner.  usage (on the GPU box, from the repo root): tools/probes/r06.sh <step>...
# Every step runs under its own time limit; the first failing step ends the call.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r06
mkdir -p $O
export TMPDIR=/tmp
ET="tools/eval_timing.py"
PT="python3 -u -m pytest -x -v --timeout 170 --timeout-method thread"
run() {  # run <seconds> <log> <cmd...>: time-limited, output appended to $O/<log>
  local t=$1 log=$2; shift 2
  echo "== $*" >> $O/$log
  timeout -k 10 "$t" "$@" >> $O/$log 2>&1 || { echo "step failed ($?): $*"; tail -40 $O/$log; exit 1; }
}
for step in "$@"; do
  case $step in
    new)    # this round's new GPU tests
      run 600 new_tests.log $PT tests/test_multigpu.py tests/test_integration_cxx.py -m gpu \
        -k "async or failure or inject" ;;
    sel)    # PYTEST_SEL="<files/-k ...>"
      run 900 sel_tests.log $PT -m gpu $PYTEST_SEL ;;
    suite)  # the whole GPU suite
      run 1000 gpu_tests.log $PT tests -m gpu ;;
    smoke)
      run 300 smoke.log python3 -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)  # the driver's default bench
      run 900 bench.log python3 bench.py && grep '^{' $O/bench.log | tail -1 > $O/bench.json ;;
    benchp) # primary line only
      run 300 benchp.log python3 bench.py --only-primary && grep '^{' $O/benchp.log | tail -1 > $O/benchp.json ;;
    h27ab)  # hex27 40^3 TotLag / linear evaluate, libraries $LIBS alternated over 2 rounds
      for rep in 1 2; do for v in $LIBS; do for k in totlag linear; do
        if [ "$v" = default ]; then unset FCG_LIB; else export FCG_LIB=$v; fi
        r=$(timeout -k 10 150 python3 $ET --celltype hex27 --kinem $k --n 40 --reps 9 | tail -1) || exit 1
        echo "$v $k $(echo "$r" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(round(d["ms_evaluate"],4), round(d["ms_element"],4), round(d["ms_assemble"],4))')" | tee -a $O/h27ab.txt
      done; done; done; unset FCG_LIB ;;
    h27pmc) # hex27 40^3 TotLag counters (mem, occ) of the element and assembly kernels, library $PLIB
      [ -n "$PLIB" ] && export FCG_LIB=$PLIB
      run 300 h27pmc.log tools/pmc_kernel.sh r06/h27pmc_${PLIB:-default}_el h27_element_kernel mem,occ -- --n 40 --celltype hex27 --kinem totlag --reps 3
      run 60 h27pmc.log python3 tools/pmc_summary.py gpurun_out/r06/h27pmc_${PLIB:-default}_el assemble27_kernel
      unset FCG_LIB ;;
    tsibis) # TSI two-field tangent (126^3) and 1M hex8 linear of the round-end builds r02..r05 and
            # HEAD, alternated over 2 rounds on this box (bisect/<r>: each round's own python + lib)
      for rep in 1 2; do for v in r02 r03 r04 r05 head; do
        d=bisect/$v; [ $v = head ] && d=.
        r=$(cd $d && timeout -k 10 200 python3 tools/tsi_bench.py --reps 20 | tail -1) || exit 1
        echo "$v tsi $r" | tee -a $O/tsibis.txt
        r=$(cd $d && timeout -k 10 120 python3 tools/eval_timing.py --n 100 --reps 40 | tail -1) || exit 1
        echo "$v lin $(echo "$r" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(round(d["ms_evaluate"],4))')" | tee -a $O/tsibis.txt
      done; done ;;
    h27occ) # hex27 40^3 element kernel at two resident workgroups per CU (default) and at one
            # (FCG_H27_DYNLDS pads the LDS), alternated over 2 rounds
      for rep in 1 2; do for v in 0 20000; do for k in totlag linear; do
        r=$(FCG_H27_DYNLDS=$v timeout -k 10 150 python3 $ET --celltype hex27 --kinem $k --n 40 --reps 9 | tail -1) || exit 1
        echo "dynlds=$v $k $(echo "$r" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(round(d["ms_evaluate"],4), round(d["ms_element"],4), round(d["ms_assemble"],4))')" | tee -a $O/h27occ.txt
      done; done; done ;;
    gpmc)   # HEAD counter sets of the gather kernel (renumbered 1M hex8, PATH_GATHER), TotLag and linear
      for k in totlag linear; do
        run 600 gpmc.log tools/pmc_kernel.sh r06/gpmc_$k gather_h8_kernel occ,inst,flop,mem -- --n 100 --renumber --path gather --kinem $k --reps 3
      done ;;
    ovlab)  # hex27 40^3 evaluate: the overlapped schedule (env knobs from $OVL_VARIANTS, "two" = the
            # two launches) alternated over 2 rounds
      for rep in 1 2; do for v in ${OVL_VARIANTS:-two default}; do for k in ${KINS:-totlag linear}; do
        envs=""; [ "$v" = two ] && envs="FCG_H27_OVERLAP=0"; [ "$v" != two ] && [ "$v" != default ] && envs="${v//,/ }"
        r=$(env $envs timeout -k 10 150 python3 $ET --celltype hex27 --kinem $k --n ${N27:-40} --reps 9 | tail -1) || exit 1
        echo "$v $k $(echo "$r" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(round(d["ms_evaluate"],4), round(d["ms_element"],4), round(d["ms_assemble"],4))')" | tee -a $O/ovlab.txt
      done; done; done ;;
    h27st)  # hex27 phase stamps (tools/h27_stamps.py, FCG_STAMPS=1), env $STENV
      run 300 h27st.log env $STENV python3 tools/h27_stamps.py ${N27:-40} ;;
    swst)   # sweep phase stamps (tools/stamps.py) and a HEAD counter set of the headline sweep
      run 300 swst.log python3 tools/stamps.py 100
      run 600 swst.log tools/pmc_kernel.sh r06/swpmc "sweep_h8_kernel<0" occ,inst,flop,mem -- --n 100 --reps 3 ;;
    libab)  # evaluate timing of libraries $LIBS (default = the product build) alternated over 2 rounds,
            # tools/eval_timing.py arguments $ETARGS, label $ABTAG
      for rep in 1 2; do for v in $LIBS; do
        if [ "$v" = default ]; then unset FCG_LIB; else export FCG_LIB=$v; fi
        r=$(timeout -k 10 150 python3 $ET $ETARGS | tail -1) || exit 1
        echo "$v $ABTAG $(echo "$r" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(round(d["ms_evaluate"],4), round(d["ms_element"],4), round(d["ms_assemble"],4))')" | tee -a $O/libab.txt
      done; done; unset FCG_LIB ;;
    tsipmc) # HEAD counter sets of the TSI split passes (126^3): the structural sweep and the thermal pass
      run 600 tsipmc.log tools/pmc_kernel.sh r06/tsipmc "sweep_h8_kernel<0, true, true, 2>" occ,inst,flop,mem -- --n 126 --tsi --reps 3
      run 60 tsipmc.log python3 tools/pmc_summary.py gpurun_out/r06/tsipmc "sweep_h8_kernel<0, true, true, 0>" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "r06 steps done: $*"
