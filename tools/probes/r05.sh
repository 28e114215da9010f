#!/bin/bash
# Round-5 GPU probe runner (one parameterised script instead of one file per gpurun call).
# usage (on the GPU box, from the repo root): tools/probes/r05.sh <step> [<step> ...]
# Every step runs under its own time limit; the first failing step ends the call.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/r05
mkdir -p $O
export TMPDIR=/tmp
ET="tools/eval_timing.py"
run() {  # run <seconds> <log> <cmd...>: time-limited, output appended to $O/<log>
  local t=$1 log=$2; shift 2
  echo "== $*" >> $O/$log
  timeout -k 10 "$t" "$@" >> $O/$log 2>&1 || { echo "step failed ($?): $*"; tail -30 $O/$log; exit 1; }
}
for step in "$@"; do
  case $step in
    h27)  # hex27 evaluate timing (element + assembly split), 40^3 linear / TotLag, 100^3 TotLag
      for k in linear totlag; do run 200 h27.jsonl python3 $ET --celltype hex27 --kinem $k --n 40 --reps 9; done
      run 300 h27.jsonl python3 $ET --celltype hex27 --kinem totlag --n 100 --reps 5
      grep '^{' $O/h27.jsonl | tail -3 ;;
    h27q)  # hex27 40^3 only
      for k in linear totlag; do run 200 h27.jsonl python3 $ET --celltype hex27 --kinem $k --n 40 --reps 9; done
      grep '^{' $O/h27.jsonl | tail -2 ;;
    slab)  # hex27 slab schedule: FCG_H27_SLAB x FCG_H27_STREAMS sweep, 40^3 TotLag / linear, 100^3 TotLag
      for k in totlag linear; do
        for sl in 0 800 1600 3200 6400; do for st in 1 2; do
          [ $sl = 0 ] && [ $st = 2 ] && continue
          echo "slab=$sl streams=$st $(FCG_H27_SLAB=$sl FCG_H27_STREAMS=$st timeout -k 10 120 python3 $ET --celltype hex27 --kinem $k --n 40 --reps 9 | tail -1)" >> $O/slab.txt || exit 1
        done; done
      done
      for sl in 0 5000 10000 20000; do for st in 1 2; do
        [ $sl = 0 ] && [ $st = 2 ] && continue
        echo "slab=$sl streams=$st $(FCG_H27_SLAB=$sl FCG_H27_STREAMS=$st timeout -k 10 300 python3 $ET --celltype hex27 --kinem totlag --n 100 --reps 5 | tail -1)" >> $O/slab.txt || exit 1
      done; done
      python3 -c "
import json
for l in open('$O/slab.txt'):
    h, j = l.split(' {', 1); d = json.loads('{' + j)
    print(h, d['config'], round(d['ms_evaluate'], 3), round(d['device_bytes'] / 1e9, 2))" ;;
    h27ab)  # same-box A/B of lib variants (FCG_LIB), hex27 40^3: h27ab with LIBS="default recw1"
      for r in 1 2; do for v in ${LIBS:-default}; do for k in linear totlag; do
        if [ "$v" = default ]; then unset FCG_LIB; else export FCG_LIB=$v; fi
        echo "$v $k $(timeout -k 10 120 python3 $ET --celltype hex27 --kinem $k --n 40 --reps 9 | tail -1)" >> $O/h27ab.txt || exit 1
      done; done; done; unset FCG_LIB
      python3 -c "
import json
for l in open('$O/h27ab.txt'):
    v, k, j = l.split(' ', 2); d = json.loads(j)
    print(v, k, round(d['ms_evaluate'], 3), round(d['ms_element'], 3), round(d['ms_assemble'], 3))" ;;
    slabprof)  # per-kernel durations of the slab schedule (rocprofv3 kernel trace)
      for sl in 0 1600 6400; do
        mkdir -p $O/slabprof_$sl
        (cd /tmp && FCG_H27_SLAB=$sl timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/slabprof_$sl" -o run -- python3 "$GRAFT_REPO_ROOT/$ET" --celltype hex27 --kinem totlag --n 40 --reps 9) > $O/slabprof_$sl.log 2>&1 || { tail -20 $O/slabprof_$sl.log; exit 1; }
        f=$(find $O/slabprof_$sl -name "*kernel_stats.csv" | head -1)
        echo "slab=$sl"; grep -E "h27_element|assemble27" "$f" | cut -d, -f1-8
      done ;;
    scratch)  # hex27 100^3 TotLag: evaluate time and ring size per slab size
      for sl in ${SLABS:-0 5000 10000 20000}; do
        echo "slab=$sl $(FCG_H27_SLAB=$sl timeout -k 10 300 python3 $ET --celltype hex27 --kinem totlag --n 100 --reps 5 | tail -1)" >> $O/scratch.txt || exit 1
      done
      python3 -c "
import json
for l in open('$O/scratch.txt'):
    h, j = l.split(' {', 1); d = json.loads('{' + j)
    print(h, round(d['ms_evaluate'], 2), 'scratch GB', round(d['scratch_bytes'] / 1e9, 3), 'device GB', round(d['device_bytes'] / 1e9, 2))" ;;
    c3)  # config 3 Newton (bench.py's secondary line): setup phases and Newton time
      run 600 c3.log env FCG_MG_SETUP_TIMING=1 FCG_MG_GRAPH_TIMING=1 python3 tools/newton_bench.py --celltype hex27 --kinem totlag --n 100 --length 1 --load -1 --mg --mg-matrix-free --mg-outer-matrix-free
      grep '^{' $O/c3.log | tail -1 > $O/c3.json
      python3 -c "
import json; d = json.load(open('$O/c3.json'))
print('setup_s', round(d['setup_s'], 2), 'newton_s', round(d['newton_s'], 3), json.dumps(d['setup_phases']))" ;;
    gab)  # same-box A/B of lib variants on the gather path: renumbered 1M hex8, LIBS="default head ..."
      for r in 1 2; do for v in ${LIBS:-default}; do for k in linear totlag; do
        if [ "$v" = default ]; then unset FCG_LIB; else export FCG_LIB=$v; fi
        echo "$v $k $(timeout -k 10 200 python3 $ET --celltype hex8 --kinem $k --n 100 --path gather --renumber --reps 9 | tail -1)" >> $O/gab.txt || exit 1
      done; done; done; unset FCG_LIB
      python3 -c "
import json
for l in open('$O/gab.txt'):
    v, k, j = l.split(' ', 2); d = json.loads(j)
    print(v, k, round(d['ms_evaluate'], 3))" ;;
    sab)  # same-box A/B of lib variants on the structured sweep: 1M hex8 linear (+ TotLag), LIBS=...
      for r in 1 2 3; do for v in ${LIBS:-default}; do for k in ${KINS:-linear}; do
        if [ "$v" = default ]; then unset FCG_LIB; else export FCG_LIB=$v; fi
        echo "$v $k $(timeout -k 10 200 python3 $ET --celltype hex8 --kinem $k --n 100 --reps 21 | tail -1)" >> $O/sab.txt || exit 1
      done; done; done; unset FCG_LIB
      python3 -c "
import json, collections
t = collections.defaultdict(list)
for l in open('$O/sab.txt'):
    v, k, j = l.split(' ', 2); d = json.loads(j); t[(v, k)].append(round(d['ms_evaluate'], 4))
for key, x in t.items(): print(key, x)" ;;
    tab)  # same-box A/B of lib variants on the TSI tangent (126^3), LIBS=...
      for r in 1 2; do for v in ${LIBS:-default}; do
        if [ "$v" = default ]; then unset FCG_LIB; else export FCG_LIB=$v; fi
        echo "$v $(timeout -k 10 300 python3 tools/tsi_bench.py --n 126 --reps 10 | tail -1)" >> $O/tab.txt || exit 1
      done; done; unset FCG_LIB
      python3 -c "
import json
for l in open('$O/tab.txt'):
    v, j = l.split(' ', 1); d = json.loads(j)
    print(v, 'split', round(d['ms_structure'], 3), '+', round(d['ms_tsi_blocks'], 3), 'fused', round(d['ms_fused'], 3))" ;;
    tsplit)  # TSI fused tangent: split (default) vs one fused pass, same box, alternating
      for r in 1 2 3; do for sp in 1 0; do
        echo "split=$sp $(FCG_TSI_SPLIT=$sp timeout -k 10 300 python3 tools/tsi_bench.py --n 126 --reps 10 | tail -1)" >> $O/tsplit.txt || exit 1
      done; done
      python3 -c "
import json
for l in open('$O/tsplit.txt'):
    v, j = l.split(' ', 1); d = json.loads(j)
    print(v, 'fused-entry', round(d['ms_fused'], 3))" ;;
    h27pmc)  # HEAD counter sets of both hex27 kernels (40^3 TotLag) and of the 1M sweep
      timeout -k 10 900 tools/pmc_kernel.sh r05/h27pmc h27_element occ,inst,flop,mem -- --celltype hex27 --kinem totlag --n 40 --reps 3 > $O/h27pmc.log 2>&1 || { tail -20 $O/h27pmc.log; exit 1; }
      python3 tools/pmc_summary.py gpurun_out/r05/h27pmc assemble27 > gpurun_out/r05/h27pmc/summary_assemble27.txt
      tail -12 gpurun_out/r05/h27pmc/summary.txt; tail -12 gpurun_out/r05/h27pmc/summary_assemble27.txt ;;
    tseg)  # TotLag sweep segmentation: the slot model at 1 / 2 / 3 / 4 workgroups per CU
      for r in 1 2 3; do for w in 1 2 3 4; do
        echo "wpc=$w $(FCG_SWEEP_TOTLAG_WGS_PER_CU=$w timeout -k 10 200 python3 $ET --celltype hex8 --kinem totlag --n 100 --reps 21 | tail -1)" >> $O/tseg.txt || exit 1
      done; done
      python3 -c "
import json, collections
t = collections.defaultdict(list)
for l in open('$O/tseg.txt'):
    v, j = l.split(' ', 1); t[v].append(round(json.loads(j)['ms_evaluate'], 4))
for k, x in t.items(): print(k, x)" ;;
    tlpmc)  # counter sets of the 1M hex8 TotLag sweep for the default build and LIBS=... variants
      for v in default ${LIBS:-}; do
        if [ "$v" = default ]; then unset FCG_LIB; else export FCG_LIB=$v; fi
        timeout -k 10 600 tools/pmc_kernel.sh r05/tlpmc_$v sweep_h8 occ,inst,flop,mem -- --celltype hex8 --kinem totlag --n 100 --reps 3 > $O/tlpmc_$v.log 2>&1 || { tail -20 $O/tlpmc_$v.log; exit 1; }
        echo "== $v"; tail -12 gpurun_out/r05/tlpmc_$v/summary.txt
      done; unset FCG_LIB ;;
    primprof)  # rocprofv3 kernel statistics of bench.py --only-primary (the headline's kernels)
      mkdir -p $O/primprof
      (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/primprof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --only-primary --steps 20 --warmup 5) > $O/primprof.log 2>&1 || { tail -20 $O/primprof.log; exit 1; }
      grep '^{' $O/primprof.log | tail -1 > $O/primprof_bench.json
      f=$(find $O/primprof -name "*kernel_stats.csv" | head -1); head -4 "$f" | cut -c1-220 ;;
    gloo2)  # bench.py --gpus 2 on one GPU over the host-staged (gloo) transport: the multi-rank flow
      FCG_DIST_BACKEND=gloo timeout -k 10 600 python -u bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --no-newton --no-amg --no-slab > $O/bench_gloo2.json 2> $O/bench_gloo2.err || { tail -20 $O/bench_gloo2.err; exit 1; }
      python3 -c "
import json; d = json.loads(open('$O/bench_gloo2.json').read().strip().splitlines()[-1])
print(d['n_gpus'], d['value'], d['ms_per_step'], d['config'])
for s in d.get('secondary', []): print(s.get('workload'), s.get('value'), s.get('error', '')[:300])" ;;
    bab)  # same-box A/B of the headline step (bench.py --only-primary): bab with LIBS="default head"
      for rep in 1 2 3; do for v in ${LIBS:-default head}; do
        if [ "$v" = default ]; then unset FCG_LIB; else export FCG_LIB=$v; fi
        timeout -k 10 300 python3 bench.py --only-primary --steps 50 --warmup 5 --no-cpu-baseline > $O/bab_$v.log 2>&1 || { tail -20 $O/bab_$v.log; exit 1; }
        echo "$v $(grep '^{' $O/bab_$v.log | tail -1)" >> $O/bab.jsonl
      done; done; unset FCG_LIB
      python3 -c "
import json
for l in open('$O/bab.jsonl'):
    v, j = l.split(' ', 1); d = json.loads(j)
    print(v, round(d['value'] / 1e6, 1), round(d['ms_per_step'], 4), round(d['roofline']['frac'], 4))" ;;
    s:*)  # one test file / node id with its prints (-s): s:tests/test_x.py::name
      run 900 gpu_tests_s.log python -u -m pytest -x -v -s --timeout 600 --timeout-method thread -m gpu "${step#s:}"
      grep -E "PASSED|FAILED|iterations|stats|passed|failed" $O/gpu_tests_s.log | cut -c1-900 | tail -40 ;;
    cxx:*)  # the C++ host's config-3 Newton (tests/cxx/config3_native N RANKS): cxx:40,2
      a=${step#cxx:}
      run 900 cxx_${a/,/_}.log tests/cxx/_build/config3_native ${a/,/ }
      tail -12 $O/cxx_${a/,/_}.log ;;
    c3lib)  # config-3 Newton, same-box A/B of lib variants: c3lib with LIBS="default x"
      for rep in 1 2; do for v in ${LIBS:-default}; do
        if [ "$v" = default ]; then unset FCG_LIB; else export FCG_LIB=$v; fi
        timeout -k 10 300 python3 tools/newton_bench.py --celltype hex27 --kinem totlag --n 100 --length 1 --load -1 --mg --mg-matrix-free --mg-outer-matrix-free > $O/c3lib_$v.log 2>&1 || { tail -20 $O/c3lib_$v.log; exit 1; }
        echo "$v $(grep '^{' $O/c3lib_$v.log | tail -1)" >> $O/c3lib.jsonl
      done; done; unset FCG_LIB
      python3 -c "
import json
for l in open('$O/c3lib.jsonl'):
    v, j = l.split(' ', 1); d = json.loads(j)
    print(v, 'newton_s', round(d['newton_s'], 3), 'solve_ms', round(d['solve_ms_total'], 1), 'asm_ms', round(d['assembly_ms_mean'], 2), 'apply_ms', round(d['tangent_apply_ms'], 3), 'its', d['pcg_iterations'])" ;;
    amglib)  # renumbered 1M hex8 TotLag Newton with the native AMG (bench.py's secondary), LIBS=...
      for rep in 1 2; do for v in ${LIBS:-default}; do
        if [ "$v" = default ]; then unset FCG_LIB; else export FCG_LIB=$v; fi
        timeout -k 10 300 python3 tools/newton_bench.py --celltype hex8 --kinem totlag --n 100 --length 1 --load=-1e-2 --renumber --amg-native > $O/amglib_$v.log 2>&1 || { tail -20 $O/amglib_$v.log; exit 1; }
        echo "$v $(grep '^{' $O/amglib_$v.log | tail -1)" >> $O/amglib.jsonl
      done; done; unset FCG_LIB
      python3 -c "
import json
for l in open('$O/amglib.jsonl'):
    v, j = l.split(' ', 1); d = json.loads(j)
    print(v, 'newton_s', round(d['newton_s'], 3), 'solve_ms', round(d['solve_ms_total'], 1), 'asm_ms', round(d['assembly_ms_mean'], 2), 'its', d['pcg_iterations'])" ;;
    rab)  # renumbered 1M hex8 through AUTO (lattice detection -> sweep MODE 3), LIBS=..., KINS=...
      for r in 1 2 3; do for v in ${LIBS:-default}; do for k in ${KINS:-linear}; do
        if [ "$v" = default ]; then unset FCG_LIB; else export FCG_LIB=$v; fi
        echo "$v $k $(timeout -k 10 300 python3 $ET --celltype hex8 --kinem $k --n 100 --renumber --reps 9 | tail -1)" >> $O/rab.txt || exit 1
      done; done; done; unset FCG_LIB
      python3 -c "
import json, collections
t = collections.defaultdict(list)
for l in open('$O/rab.txt'):
    v, k, j = l.split(' ', 2); d = json.loads(j); t[(v, k)].append(round(d['ms_evaluate'], 4))
for key, x in t.items(): print(key, x)" ;;
    tests)  # the whole GPU suite
      run 1500 gpu_tests.log python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests
      tail -3 $O/gpu_tests.log ;;
    t:*)  # one test file / node id: t:tests/test_x.py::name
      run 900 gpu_tests_part.log python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "${step#t:}"
      tail -3 $O/gpu_tests_part.log ;;
    bench)
      run 900 bench.log python3 bench.py --gpus 1 --steps 20 --warmup 5
      grep '^{' $O/bench.log | tail -1 > $O/bench.json ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
