"""Benchmark: element evaluations/s and global-assembly wall time of 4C's SOLID hex8 linear
elasticity path (BASELINE.json config 2: 1M hex8 per GPU, K and r assembled) on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W]      (N > 1: starts its N ranks itself)
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (one rank per GPU)

Without WORLD_SIZE in the environment, `--gpus N` (N > 1) starts N rank processes of this script
(tools/rank_launcher.py: RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*, before torch is imported, no
exec) and exits with the first failing rank's code; under a launcher WORLD_SIZE must equal N.

One step = Discretization::set_state (row -> column import of the displacement; RCCL all-to-all
of the ghost DOFs when N > 1) + Discretization::evaluate(struct_calc_nlnstiff) with zero() fused
(K and f_int of the rank's owned rows written once).  The K timed steps are queued back to back and
the element-error flags (4C's throws) are read once after them, inside the window.  The residual
norm (NOX's Norm2 -> all-reduce) is a Newton-loop ingredient outside the assembly window since
round 3: it is timed per step in a separate pass (ranks[].ms_norm_allreduce), and
`ms_per_step_with_norm` = ms_per_step + that time is the figure comparable with rounds 1-2, whose
step included the norm and a flag read per step.
Weak scaling: every rank owns a 100^3 hex8 box of the GridGenerator split (N=8 -> 200^3, 8M).
Inputs (mesh, u) are resident in HBM before the timed region.  Synthetic data: grid-generator box
[0,1]^3 scaled per rank count, interior jitter 0.1h (SplitMix64 seed 20251015),
u = 1e-3 (sin2piX cospiY, sinpiY cos2piZ, sin2piZ cospiX), StVK E=210 nu=0.3.
"""

import argparse
import glob
import json
import os
import platform
import re
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import rank_launcher  # noqa: E402  (standard library only)

if __name__ == "__main__":
    # one process per GPU: start the ranks here, before anything can initialise HIP
    rank_launcher.run_or_spawn(sys.argv, os.path.abspath(__file__))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

sys.path.insert(0, ROOT)

import importlib  # noqa: E402

pkg = importlib.import_module("4c_amd")
fcg = pkg.fcg
halo = importlib.import_module("4c_amd.halo")

HBM_PEAK_GBS = 8000.0     # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
FP64_PEAK_TFS = 78.6      # MI355X FP64 vector (= matrix) spec, SURVEY.md §8d
# SURVEY.md §8d algorithmic figures for hex8 linear K + r (per element)
ALG_BYTES_PER_ELE = 2069.0
ALG_FLOP_PER_ELE = 41.4e3


def _gridgen_subdivisions(iv, world):
    """Processor grid of GridGenerator's box split (4C_io_gridgenerator.cpp:87-117): prime
    factors, largest first, each to the direction with the largest interval per subdivision."""
    factors, w, f = [], world, 2
    while w > 1:
        if w % f == 0:
            factors.append(f)
            w //= f
        else:
            f += 1
    sub = [1, 1, 1]
    for fac in reversed(factors):
        r = [iv[d] / sub[d] for d in range(3)]
        d = 0 if (r[0] >= r[1] and r[0] >= r[2]) else (1 if r[1] >= r[2] else 2)
        sub[d] *= fac
    return sub


def weak_interval(n, world):
    """Global INTERVALS such that GridGenerator's own split gives every rank an n^3 box: the
    processor grid as cubic as the prime factors allow (N=8 -> 2x2x2, i.e. config 4's 200^3),
    checked against the reference's split rule; slabs along x otherwise."""
    factors, w, f = [], world, 2
    while w > 1:
        if w % f == 0:
            factors.append(f)
            w //= f
        else:
            f += 1
    p = [1, 1, 1]
    for fac in reversed(factors):
        d = int(np.argmin(p))
        p[d] *= fac
    iv = tuple(n * p[d] for d in range(3))
    if _gridgen_subdivisions(iv, world) == p:
        return iv
    return (n * world, n, n)


def cpu_baseline(n, kinem, threads):
    """Oracle (4C-faithful restatement, oracle/) on the host cores: reference MPI semantics with
    `threads` workers as ranks, each assembling its own rows.  Bounded sample: one evaluation of
    the full n^3 mesh (about 10-30 s of CPU work in total)."""
    parity_util = _oracle_native()
    mesh = fcg.BoxMesh(fcg.HEX8, (n, n, n), jitter=0.1, seed=20251015)
    u = mesh.u_col(1e-3)
    # single-core rate on a small slab, then all-core on the full mesh
    small = fcg.BoxMesh(fcg.HEX8, (n, n, max(2, n // 20)), jitter=0.1, seed=20251015)
    us = small.u_col(1e-3)
    t = time.perf_counter()
    parity_util.oracle_evaluate(small, kinem, 210.0, 0.3, us, nworkers=1)
    t1 = time.perf_counter() - t
    t = time.perf_counter()
    err, _, _, _ = parity_util.oracle_evaluate(mesh, kinem, 210.0, 0.3, u, nworkers=threads)
    tn = time.perf_counter() - t
    assert err == 0
    # thread scaling on the full mesh, measured up to the granted share (the GridGenerator split
    # into t ranks, each assembling its own rows): backs the all-core extrapolation below
    scaling = {"1 (slab)": small.n_ele / t1, str(threads): mesh.n_ele / tn}
    tc = max(2, threads // 4)
    while tc < threads:
        t = time.perf_counter()
        parity_util.oracle_evaluate(mesh, kinem, 210.0, 0.3, u, nworkers=tc)
        scaling[str(tc)] = mesh.n_ele / (time.perf_counter() - t)
        tc *= 2
    try:
        model = [l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")][0]
    except Exception:
        model = platform.processor()
    topo = cpu_topology()
    phys = topo.get("physical_cores") or threads
    return {
        "value": mesh.n_ele / tn, "unit": "element-evaluations/s", "cores": threads,
        "kind": "port",
        "sample": f"one struct_calc_nlnstiff evaluation of the full {n}^3 hex8 mesh "
                  f"({mesh.n_ele} elements, K+r assembled), {threads} threads as ranks (the CPU "
                  f"share granted to this process); single-core {small.n_ele / t1:.4g} elem/s on "
                  f"{small.n_ele} elements",
        "wall_s": tn, "single_core_value": small.n_ele / t1, "cpu_model": model,
        "topology": topo,
        "thread_scaling_measured": scaling,
        "parallel_efficiency_measured": (mesh.n_ele / tn) / (threads * small.n_ele / t1),
        # not measured: the GPU box grants this process `threads` CPUs (OMP_NUM_THREADS; the
        # other cores belong to other GPUs' jobs), so the all-core figure is the single-core rate
        # times every physical core at the parallel efficiency measured at `threads`
        "all_physical_cores_extrapolated": small.n_ele / t1 * phys
                                           * min(1.0, (mesh.n_ele / tn) / (threads * small.n_ele / t1)),
        "all_cores_note": "not run: the box's CPU share for one GPU is the granted thread count; "
                          "extrapolated from the measured single-core rate and scaling",
        "compiler": "gcc -O3 -march=native -fopenmp",
    }


def _pmc_key(path):
    """(round, version) of profiles/pmc_rNN[_vM].json; older files sort first."""
    m = re.search(r"pmc_r(\d+)(?:_v(\d+))?\.json$", os.path.basename(path))
    return (int(m.group(1)), int(m.group(2) or 0)) if m else (-1, -1)


def committed_pmc(explicit=None):
    """The committed PMC traffic file: `explicit`, else the newest by (round, version)."""
    if explicit:
        return explicit
    files = glob.glob(os.path.join(ROOT, "profiles", "pmc_r*.json"))
    return max(files, key=_pmc_key) if files else None


def _under_profiler():
    pre = os.environ.get("LD_PRELOAD", "") + os.environ.get("HSA_TOOLS_LIB", "")
    return "rocprof" in pre or any(k.startswith("ROCPROF") for k in os.environ)


def measure_counters(passes, prof_args, kernel, timeout_s=150):
    """Per-dispatch means of rocprofv3 counters for the kernels whose name contains `kernel`,
    measured in this run: one child process per pass (tools/prof_kernel.py `prof_args`, a few
    evaluates of the workload), each under its own time limit and with no tracing domain mixed in.
    Returns {counter: mean per dispatch} (or a dict with "error")."""
    import csv
    import shutil
    import tempfile
    rp = shutil.which("rocprofv3")
    if rp is None:
        return {"error": "rocprofv3 not found"}
    if _under_profiler():
        return {"error": "bench.py is itself running under a profiler: no nested counter passes"}
    work = tempfile.mkdtemp(prefix="fcg_pmc_")
    per = {}
    try:
        for i, ctrs in enumerate(passes):
            d = os.path.join(work, f"p{i}")
            cmd = [rp, "--pmc", *ctrs.split(), "--output-format", "csv", "-d", d, "-o", "run", "--",
                   sys.executable, os.path.join(ROOT, "tools", "prof_kernel.py"), *prof_args]
            env = dict(os.environ, TMPDIR=work)
            p = subprocess.run(cmd, cwd=work, env=env, capture_output=True, text=True,
                               timeout=timeout_s)
            if p.returncode != 0:
                return {"error": f"pass {ctrs} exited {p.returncode}: {p.stderr[-400:]}"}
            vals = {}
            for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
                for r in csv.DictReader(open(fn)):
                    if kernel in r["Kernel_Name"]:
                        key = (r["Counter_Name"], r["Dispatch_Id"])
                        vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
            for c in ctrs.split():
                v = [x for (name, _), x in vals.items() if name == c]
                if not v:
                    return {"error": f"{c}: no {kernel} dispatch in the counter output"}
                per[c] = sum(v) / len(v)
        return per
    except subprocess.TimeoutExpired:
        return {"error": f"counter pass exceeded {timeout_s} s"}
    finally:
        shutil.rmtree(work, ignore_errors=True)


def measure_mfma_h27(n, cus):
    """Matrix-pipe use of h27_element_kernel on the config-3 element box, measured in this run:
    SQ_VALU_MFMA_BUSY_CYCLES (summed over the SIMDs) against the SIMD-cycles of the dispatch
    (GRBM_GUI_ACTIVE summed over the 8 XCDs -> / 8 per XCD, x 4 SIMDs x CUs), and the FP64 MFMA
    flops it executed (SQ_INSTS_VALU_MFMA_F64 x 2048 for v_mfma_f64_16x16x4_f64)."""
    c = measure_counters(["SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 "
                          "SQ_INSTS_VALU_FLOPS_FP64 GRBM_GUI_ACTIVE"],
                         ["--n", str(n), "--celltype", "hex27", "--kinem", "totlag", "--reps", "3"],
                         "h27_element_kernel")
    if "error" in c:
        return c
    simd_cycles = c["GRBM_GUI_ACTIVE"] / 8.0 * 4.0 * cus
    return {"mfma_busy_cycles": c["SQ_VALU_MFMA_BUSY_CYCLES"], "simd_cycles": simd_cycles,
            "matrix_pipe_busy_frac": c["SQ_VALU_MFMA_BUSY_CYCLES"] / simd_cycles,
            "mfma_f64_instructions": c["SQ_INSTS_VALU_MFMA_F64"],
            "mfma_f64_mops": c["SQ_INSTS_VALU_MFMA_MOPS_F64"],
            "mfma_f64_flop_per_evaluate": 2048.0 * c["SQ_INSTS_VALU_MFMA_F64"],
            "valu_flops_fp64_counter": c["SQ_INSTS_VALU_FLOPS_FP64"],
            "source": "measured in this run: rocprofv3 --pmc (one child pass of tools/prof_kernel.py, "
                      "3 evaluates, mean per dispatch)"}


def measure_traffic(n, kernel="sweep_h8", timeout_s=150, extra=()):
    """HBM bytes per evaluate of the bench kernel, measured in this run: two rocprofv3 counter
    passes (FETCH_SIZE, then WRITE_SIZE -- they do not fit one pass), each a child process
    (tools/prof_kernel.py: the same n^3 mesh, seed and kernel, 3 evaluates) under its own time
    limit.  Corrections of MI355X_MICROARCH.md "HBM": counters in KiB, gfx950 FETCH_SIZE counts
    half the bytes of wide reads (x2), WRITE_SIZE exact.  Returns a dict (or one with "error")."""
    import csv
    import shutil
    import tempfile
    rp = shutil.which("rocprofv3")
    if rp is None:
        return {"error": "rocprofv3 not found"}
    if _under_profiler():
        return {"error": "bench.py is itself running under a profiler: no nested counter passes"}
    work = tempfile.mkdtemp(prefix="fcg_pmc_")
    per = {}
    try:
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(work, ctr)
            cmd = [rp, "--pmc", ctr, "--output-format", "csv", "-d", d, "-o", "run", "--",
                   sys.executable, os.path.join(ROOT, "tools", "prof_kernel.py"), "--n", str(n),
                   "--seed", "20251015", "--reps", "3", *extra]
            env = dict(os.environ, TMPDIR=work)
            p = subprocess.run(cmd, cwd=work, env=env, capture_output=True, text=True,
                               timeout=timeout_s)
            if p.returncode != 0:
                return {"error": f"{ctr} pass exited {p.returncode}: {p.stderr[-400:]}"}
            vals = {}
            for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
                for r in csv.DictReader(open(fn)):
                    if kernel in r["Kernel_Name"] and r["Counter_Name"] == ctr:
                        vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
            if not vals:
                return {"error": f"{ctr}: no {kernel} dispatch in the counter output"}
            per[ctr] = sum(vals.values()) / len(vals)
        fetch = 2.0 * 1024.0 * per["FETCH_SIZE"]
        write = 1024.0 * per["WRITE_SIZE"]
        return {"fetch_bytes_x2": fetch, "write_bytes": write, "hbm_bytes_per_evaluate": fetch + write,
                "source": "measured in this run: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate "
                          "child passes of tools/prof_kernel.py (3 evaluates, mean per dispatch)"}
    except subprocess.TimeoutExpired:
        return {"error": f"counter pass exceeded {timeout_s} s"}
    finally:
        shutil.rmtree(work, ignore_errors=True)


def cpu_threads(requested):
    """Threads of the CPU baseline: the CPU share this process may use (the affinity mask; on the
    GPU box the harness grants 16 CPUs per GPU and exports OMP_NUM_THREADS accordingly)."""
    if requested > 0:
        return requested
    share = len(os.sched_getaffinity(0))
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return max(1, min(share, omp) if omp > 0 else share)


def cpu_topology():
    """nproc, physical cores and SMT state of the host (lscpu semantics from /sys)."""
    out = {"nproc_affinity": len(os.sched_getaffinity(0)), "logical_cpus": os.cpu_count()}
    try:
        cores = set()
        base = "/sys/devices/system/cpu"
        for d in os.listdir(base):
            if d.startswith("cpu") and d[3:].isdigit():
                try:
                    pk = open(f"{base}/{d}/topology/physical_package_id").read().strip()
                    co = open(f"{base}/{d}/topology/core_id").read().strip()
                    cores.add((pk, co))
                except OSError:
                    pass
        out["physical_cores"] = len(cores) or None
        out["smt_active"] = open(f"{base}/smt/active").read().strip() == "1"
    except OSError:
        pass
    return out


# the matrix-free hex27 action (fcg_tangent_apply) per element and application, algorithmic
# bytes: the element's 27 nodes' X, u and x (3 x 81 doubles) and 27 DOF column indices read, the
# 81 incidence values written and read back once by the row-node sum, 81 values of y written
# (every value counted once per element: the minimum traffic of an element-by-element action
# without cross-element reuse)
ALG_BYTES_PER_ELE_H27_APPLY = 8.0 * 3 * 81 + 4.0 * 27 + 8.0 * 81 * 2 + 8.0 * 81


def newton_secondary(n, timeout_s=900, cpu_rate=None):
    """BASELINE config 3: StVK TotLag on the 1M-hex27 cube (x- clamped, traction -1 in z on x+),
    full static Newton on this GPU (fcg_evaluate_device + Dirichlet + multigrid-preconditioned
    flexible CG, 4c_amd/newton.py + multigrid.py; the fine level's smoother and the outer FCG apply
    the Dirichlet-modified tangent K(u) element by element, fcg_tangent_apply -- the assembled K,
    formed every Newton step, sets the block-Jacobi smoother and equals that action at 1e-13 --
    same FCG iterations and tip displacement as with the assembled outer operator, profiles/r04/
    r04_config3_newton_outer_*.json), run by tools/newton_bench.py in
    a child process so that its ~60 GB of device buffers are released when it ends."""
    cmd = [sys.executable, os.path.join(ROOT, "tools", "newton_bench.py"), "--celltype", "hex27",
           "--kinem", "totlag", "--n", str(n), "--length", "1", "--load", "-1", "--mg",
           "--mg-matrix-free", "--mg-outer-matrix-free"]
    t = time.perf_counter()
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout_s)
    wall = time.perf_counter() - t
    if p.returncode != 0:
        return {"workload": f"hex27-totlag-{n}^3-newton", "error": p.stderr[-2000:]}
    d = json.loads(p.stdout.strip().splitlines()[-1])
    if not d.get("converged"):
        return {"workload": f"hex27-totlag-{n}^3-newton", "error": "Newton did not converge"}
    out = {
        "workload": f"hex27-totlag-{n}^3-full-newton",
        "baseline_config": "BASELINE.json configs[2] (StVK, 1M hex27, full Newton loop on 1 MI355X)",
        "value": d["newton_s"], "unit": "s (Newton loop, setup excluded)", "higher_is_better": False,
        "newton_iterations": d["newton_iterations"], "linear_iterations": d["pcg_iterations"],
        "linear_solver": d["linear_solver"], "forcing": d["forcing"],
        "norm_res": [h["norm_res"] for h in d["history"]],
        "assembly_ms_mean": d["assembly_ms_mean"], "assembly_elem_per_s": d["assembly_elem_per_s"],
        "solve_ms_total": d["solve_ms_total"], "setup_s": d["setup_s"],
        "setup_phases": d.get("setup_phases"), "wall_s": wall,
        "elements": d["elements"], "dofs": d["dofs"], "nnz": d["nnz"], "tip_uz": d["tip_uz"],
        "h27_slabs": d.get("h27_slabs"), "scratch_bytes": d.get("scratch_bytes"),
        "tangent_symmetry_rel": d.get("tangent_symmetry_rel"),
    }
    # the loop's two device phases against the HBM roof: the K + r assembly of every Newton
    # iteration (SURVEY §8d's 37,695 B per hex27 element) and the matrix-free tangent action the
    # solve applies (ALG_BYTES_PER_ELE_H27_APPLY per element)
    ne = d["elements"]
    asm = float(np.median(d["assembly_ms"])) if d.get("assembly_ms") else d["assembly_ms_mean"]
    gbs = ALG_BYTES_PER_ELE_H27 * ne / (asm * 1e-3) / 1e9
    rl = {"bound": "hbm", "kernel": "assembly: h27_element_kernel + assemble27_kernel",
          "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
          "alg_bytes_per_element": ALG_BYTES_PER_ELE_H27, "ms_assembly_median": asm}
    if d.get("tangent_apply_ms"):
        ag = ALG_BYTES_PER_ELE_H27_APPLY * ne / (d["tangent_apply_ms"] * 1e-3) / 1e9
        rl["tangent_apply"] = {"kernel": "h27_apply_sf_kernel + h27_inc_sum_kernel (fcg_tangent_apply)",
                               "ms": d["tangent_apply_ms"], "achieved": ag, "unit": "GB/s",
                               "frac": ag / HBM_PEAK_GBS,
                               "alg_bytes_per_element": ALG_BYTES_PER_ELE_H27_APPLY}
    out["roofline"] = rl
    if cpu_rate:
        # the CPU leg: the oracle's K + r assembly rate of the hex27 line (a bounded slab), scaled
        # to this loop's assemblies; the reference's CPU solve (Belos + MueLu, not vendored) has no
        # counterpart in the oracle and is not timed
        nasm = len(d.get("assembly_ms") or []) or (d["newton_iterations"] + 1)
        out["cpu_baseline"] = dict(cpu_rate, kind="port",
                                   assembly_s_per_newton_loop_extrapolated=nasm * ne / cpu_rate["value"],
                                   note="assembly only: the oracle has no CPU linear solve")
    return out


def amg_newton_secondary(n, timeout_s=600):
    """The 1M-hex8 box renumbered as an input-file mesh (no lattice hint), x- clamped,
    tip load, StVK TotLag full Newton with the native smoothed-aggregation AMG object
    (fcg_amg_create / fcg_amg_solve) -- the solve 4C's MueLu does on meshes without a box --
    run by tools/newton_bench.py in a child process."""
    cmd = [sys.executable, os.path.join(ROOT, "tools", "newton_bench.py"), "--celltype", "hex8",
           "--kinem", "totlag", "--n", str(n), "--length", "1", "--load=-1e-2", "--renumber",
           "--amg-native"]
    t = time.perf_counter()
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout_s)
    wall = time.perf_counter() - t
    name = f"hex8-totlag-{n}^3-renumbered-full-newton-amg"
    if p.returncode != 0:
        return {"workload": name, "error": p.stderr[-2000:]}
    d = json.loads(p.stdout.strip().splitlines()[-1])
    if not d.get("converged"):
        return {"workload": name, "error": "Newton did not converge"}
    out = {
        "workload": name,
        "baseline_config": "BASELINE.json configs[1] mesh without lattice, full Newton (SURVEY §8f row 2)",
        "value": d["newton_s"], "unit": "s (Newton loop, setup excluded)", "higher_is_better": False,
        "newton_iterations": d["newton_iterations"], "linear_iterations": d["pcg_iterations"],
        "linear_solver": d["linear_solver"], "amg_levels": d["mg_levels"],
        "amg_numeric_setup_ms": d["amg_numeric_setup_ms"], "amg_graph_setup_s": d["amg_graph_setup_s"],
        "assembly_ms_mean": d["assembly_ms_mean"], "solve_ms_total": d["solve_ms_total"],
        "norm_res": [h["norm_res"] for h in d["history"]], "wall_s": wall,
        "elements": d["elements"], "dofs": d["dofs"], "nnz": d["nnz"],
        "setup_phases": d.get("setup_phases"),
    }
    # the K + r assembly of each Newton iteration (node-row gather, TotLag) against the HBM roof,
    # SURVEY §8d's 2,069 B per hex8 element
    asm = float(np.median(d["assembly_ms"])) if d.get("assembly_ms") else d["assembly_ms_mean"]
    gbs = ALG_BYTES_PER_ELE * d["elements"] / (asm * 1e-3) / 1e9
    out["roofline"] = {"bound": "hbm", "kernel": "assembly: gather_h8_kernel<TotLag>",
                       "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                       "frac": gbs / HBM_PEAK_GBS, "alg_bytes_per_element": ALG_BYTES_PER_ELE,
                       "ms_assembly_median": asm}
    return out


# SURVEY.md §8d algorithmic figures for hex27 TotLag K + r (per element)
ALG_BYTES_PER_ELE_H27 = 37695.0
ALG_FLOP_PER_ELE_H27_TOTLAG = 2.59e6
# flops the hex27 kernel (fcg_hex27.hip, reference-coordinate contracted form) executes per
# TotLag element, useful work only (no MFMA padding): J and du/dxi 162 x 27 x 3 FMA; w, v per
# (g, a) 729 x 18; H + geo of the 378 pairs a <= b 378 x 27 x 12; q and f_e 2 x 729 x 9; G on the
# matrix cores 378 x 27 x 9 -- 253.8k FMA = 507.6k flop -- plus ~20k flop of Gauss-point algebra
# and block assembly
EXEC_FLOP_PER_ELE_H27_TOTLAG = 2.0 * (162 * 27 * 3 + 729 * 18 + 378 * 27 * 12 + 2 * 729 * 9
                                      + 378 * 27 * 9) + 2.0e4


def _oracle_native():
    """The oracle (oracle/) compiled -O3 -march=native for the host cores (CPU baseline leg only)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib
    import tempfile
    out = os.path.join(tempfile.gettempdir(), f"liborc_native_{os.getpid()}.so")
    if oracle_lib._lib is None or getattr(oracle_lib, "_native_out", None) != out:
        oracle_lib.build(force=True, extra_flags=["-march=native"], out=out)
        oracle_lib._lib = None
        oracle_lib._lib = oracle_lib.load(out)
        oracle_lib._native_out = out
    import parity_util
    return parity_util


def hex27_secondary(dev, n, steps, threads, with_cpu):
    """BASELINE config 3's element (hex27, StVK, TotLag, state A = 5e-2) on one GPU: K + r
    assembly rate on an n^3 box (the per-element rate is flat from 40^3 up; the 1M-element Newton
    loop itself is tools/newton_bench.py, profiles/r01_config3_hex27_1M_totlag_newton.json), the
    FP64 and HBM fractions with SURVEY §8d's per-element figures, and the oracle beside it."""
    mesh = fcg.BoxMesh(fcg.HEX27, (n, n, n), jitter=0.02, seed=20251015)
    ev = fcg.Evaluator(mesh, kinematics=fcg.TOTLAG, youngs=210.0, poisson=0.3, device=dev.index)
    u_h = mesh.u_col(5e-2)
    u = torch.from_numpy(u_h).to(dev)
    f = torch.zeros(mesh.n_rows, dtype=torch.float64, device=dev)
    K = torch.zeros(mesh.nnz, dtype=torch.float64, device=dev)
    for _ in range(2):
        ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, u, f, K)
    ev.set_timing(True)
    ts = []
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, u, f, K)
        ts.append(ev.timing())
    torch.cuda.synchronize(dev)
    wall = (time.perf_counter() - t0) / steps
    ms_kern = float(np.mean([a + b for a, b in ts]))
    flops = EXEC_FLOP_PER_ELE_H27_TOTLAG * mesh.n_ele / (ms_kern * 1e-3) / 1e12
    flops_survey = ALG_FLOP_PER_ELE_H27_TOTLAG * mesh.n_ele / (ms_kern * 1e-3) / 1e12
    gbs = ALG_BYTES_PER_ELE_H27 * mesh.n_ele / (ms_kern * 1e-3) / 1e9
    out = {
        "workload": f"hex27-totlag-{n}^3", "baseline_config": "BASELINE.json configs[2] element",
        "value": mesh.n_ele / wall, "unit": "element-evaluations/s", "ms_per_step": 1e3 * wall,
        "elements": mesh.n_ele, "nnz": mesh.nnz, "h27_slabs": int(ev.info.h27_slabs),
        "path": ("general: h27_element_kernel (two elements in flight per workgroup: wave 3 forms "
                 "the next element's Jacobians (MFMA) and Gauss-point factors while waves 0-2 put "
                 "this one's G, c_ab, geo on v_mfma_f64_16x16x4_f64) writing the owned incidences' "
                 "block rows + assemble27_kernel (one contiguous row write per node)"),
        # bound by the flops the kernel executes (507.6k FMA-flop + ~20k per element, the
        # reference-coordinate contracted form; EXEC_FLOP_PER_ELE_H27_TOTLAG) against the 37.7 kB
        # of HBM: 6.7 ns vs 4.7 ns per element at the spec peaks -> FP64 (matrix = vector peak)
        "roofline": {"bound": "fp64", "achieved": flops, "peak": FP64_PEAK_TFS, "unit": "TFLOP/s",
                     "frac": flops / FP64_PEAK_TFS, "exec_flop_per_element": EXEC_FLOP_PER_ELE_H27_TOTLAG,
                     "survey_flop_per_element": ALG_FLOP_PER_ELE_H27_TOTLAG,
                     "survey_count_tflops": flops_survey,
                     "hbm_achieved_gbs": gbs, "hbm_frac": gbs / HBM_PEAK_GBS,
                     "alg_bytes_per_element": ALG_BYTES_PER_ELE_H27,
                     "ms_element_kernel": float(np.mean([a for a, _ in ts])),
                     "ms_assemble_kernel": float(np.mean([b for _, b in ts]))},
    }
    ev.close()
    del K, f, u
    # matrix-pipe use of the element kernel (north_star: "MFMA utilisation reported against gfx950
    # peak"), from counters of this run, beside the executed-flop fraction above
    ms_el = out["roofline"]["ms_element_kernel"]
    mf = measure_mfma_h27(n, torch.cuda.get_device_properties(dev).multi_processor_count)
    if "error" not in mf:
        mf["mfma_tflops"] = mf["mfma_f64_flop_per_evaluate"] / (ms_el * 1e-3) / 1e12
        mf["mfma_frac_of_spec_fp64"] = mf["mfma_tflops"] / FP64_PEAK_TFS
    out["roofline"]["mfma_counters"] = mf
    if with_cpu:
        pu = _oracle_native()
        small = fcg.BoxMesh(fcg.HEX27, (n, n, max(2, n // 10)), jitter=0.02, seed=20251015)
        us = small.u_col(5e-2)
        t = time.perf_counter()
        err, _, _, _ = pu.oracle_evaluate(small, fcg.TOTLAG, 210.0, 0.3, us, nworkers=threads)
        tn = time.perf_counter() - t
        assert err == 0
        out["cpu_baseline"] = {"value": small.n_ele / tn, "unit": "element-evaluations/s",
                               "cores": threads, "kind": "port",
                               "sample": f"one struct_calc_nlnstiff evaluation (K + r) of a "
                                         f"{n}x{n}x{max(2, n // 10)} hex27 TotLag slab, "
                                         f"{threads} threads as ranks"}
    return out


def hex27_slab_secondary(dev, n, steps, slab):
    """Config 3's mesh (n^3 hex27, StVK TotLag) assembled under the slab schedule of the incidence
    records: the records live in a ring instead of one per incidence -- the memory
    mode for meshes whose full scratch would not fit beside the tangent.  Same K and f bitwise as
    the one-slab path (tests/test_h27_slab.py); reported: time per evaluate and the bytes."""
    os.environ["FCG_H27_SLAB"] = str(slab)
    try:
        mesh = fcg.BoxMesh(fcg.HEX27, (n, n, n), jitter=0.02, seed=20251015)
        ev = fcg.Evaluator(mesh, kinematics=fcg.TOTLAG, youngs=210.0, poisson=0.3, device=dev.index)
    finally:
        del os.environ["FCG_H27_SLAB"]
    info = ev.info
    u = torch.from_numpy(mesh.u_col(5e-2)).to(dev)
    f = torch.zeros(mesh.n_rows, dtype=torch.float64, device=dev)
    K = torch.zeros(mesh.nnz, dtype=torch.float64, device=dev)
    ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, u, f, K)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, u, f, K)
    torch.cuda.synchronize(dev)
    ms = 1e3 * (time.perf_counter() - t0) / steps
    full = int(info.n_incidences) * (9 * 27 + 3) * 8
    out = {"workload": f"hex27-totlag-{n}^3-slab-schedule",
           "baseline_config": "BASELINE.json configs[2] mesh, incidence records in a ring",
           "value": mesh.n_ele / (ms * 1e-3), "unit": "element-evaluations/s", "ms_per_step": ms,
           "slab_elements": slab, "h27_slabs": int(info.h27_slabs),
           "scratch_bytes": int(info.scratch_bytes),
           "scratch_bytes_one_record_per_incidence": full, "device_bytes": int(info.device_bytes),
           "tangent_bytes": 8 * mesh.nnz}
    ev.close()
    del K, f, u
    return out


def tsi_cpu_baseline(n, nz, threads):
    """The oracle's TSI::Monolithic element loop (orc_tsi_discretization_evaluate: the four
    blocks and both residuals, owned rows, `threads` workers as ranks) on an n x n x nz slab of the
    config-5 box, timed on the host cores."""
    pu = _oracle_native()
    E, NU, ALPHA, T0, COND, DT = 210.0, 0.3, 1.2e-5, 293.0, 52.0, 0.5
    m = fcg.BoxMesh(fcg.HEX8, (n, n, nz), upper=(1.0, 1.0, nz / n), jitter=0.1, seed=20251015)
    g = fcg.TsiGraph(m)
    X = m.node_x
    Tn = T0 + 50.0 * np.sin(2 * np.pi * X[:, 0]) * np.cos(np.pi * X[:, 1])
    t = time.perf_counter()
    err = pu.oracle_tsi_evaluate(m, g, E, NU, ALPHA, T0, COND, 1.0, 1.0 / DT, m.u_col(1e-3),
                                 m.u_col(1e-2), Tn, nworkers=threads)[0]
    tn = time.perf_counter() - t
    assert err == 0
    return {"value": m.n_ele / tn, "unit": "element-evaluations/s (two-field tangent)",
            "cores": threads, "kind": "port",
            "sample": f"one TSI two-field tangent (K_SS, k_ST, k_TS, k_TT, f_S, f_T) of a {n}x{n}x{nz} "
                      f"slab of the 126^3 box ({m.n_ele} elements), {threads} threads as ranks",
            "wall_s": tn}


def tsi_secondary(dev, rank, world, steps, n=126, cpu_threads_=0):
    """BASELINE config 5: the monolithic TSI two-field tangent (K_SS, k_ST, k_TS, k_TT, f_S, f_T;
    hex8, geometrically linear ThermoStVenantKirchhoff + Fourier) of a 126^3 = 2M-element box,
    strong-scaled: every rank assembles its GridGenerator share (owned rows, ghost layer, no
    communication) with the fused structured sweep (fcg_tsi_evaluate_fused).  Every rank makes
    the same collective calls whatever happens locally (one barrier, one max all-reduce)."""
    E, NU, ALPHA, T0, COND, DT = 210.0, 0.3, 1.2e-5, 293.0, 52.0, 0.5
    err, held, t_setup = None, None, time.perf_counter()
    try:
        m = fcg.BoxMesh(fcg.HEX8, (n, n, n), jitter=0.1, seed=20251015, rank=rank, nranks=world)
        ev = fcg.Evaluator(m, kinematics=fcg.LINEAR, youngs=E, poisson=NU, device=dev.index,
                           path=fcg.PATH_STRUCTURED)
        tev = fcg.TsiEvaluator(m, E, NU, ALPHA, T0, COND, device=dev.index)
        g = tev.graph
        X = m.node_x
        T_h = np.empty(g.n_cols_t)
        T_h[g.node_dof_col_t] = T0 + 50.0 * np.sin(2 * np.pi * X[:, 0]) * np.cos(np.pi * X[:, 1])
        f64 = dict(dtype=torch.float64, device=dev)
        T = torch.from_numpy(T_h).to(dev)
        u = torch.from_numpy(m.u_col(1e-3)).to(dev)
        v = torch.from_numpy(m.u_col(1e-2)).to(dev)
        bufs = dict(fs=torch.zeros(m.n_rows, **f64), Kss=torch.zeros(m.nnz, **f64),
                    Kst=torch.zeros(g.nnz_st, **f64), Kts=torch.zeros(g.nnz_ts, **f64),
                    Ktt=torch.zeros(g.nnz_tt, **f64), fT=torch.zeros(g.n_rows_t, **f64))
        held = (m, ev, tev, u, v, T, bufs)
        for _ in range(2):
            tev.evaluate_fused(ev, fcg.OVERWRITE, u, v, T, 1.0, 1.0 / DT, **bufs)
        torch.cuda.synchronize(dev)
    except Exception as e:  # reported below, after the same collectives as the other ranks
        err = e
    t_setup = time.perf_counter() - t_setup
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    if err is None:
        try:
            m, ev, tev, u, v, T, bufs = held
            for _ in range(steps):
                tev.evaluate_fused(ev, fcg.OVERWRITE, u, v, T, 1.0, 1.0 / DT, **bufs)
            torch.cuda.synchronize(dev)
        except Exception as e:
            err = e
    t = time.perf_counter() - t0
    res = torch.tensor([t, 1.0 if err is not None else 0.0], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(res, op=dist.ReduceOp.MAX)
    if err is not None or res[1].item() != 0.0:
        return {"workload": f"tsi-hex8-linear-{n}^3", "error": repr(err) if err else "another rank failed"}
    wall = res[0].item() / steps
    m, ev, tev, u, v, T, bufs = held
    g = tev.graph
    byt = 8 * (m.nnz + g.nnz_st + g.nnz_ts + g.nnz_tt + m.n_rows + g.n_rows_t) + 8 * 10 * m.n_node
    gbs = byt / wall / 1e9
    out = {"workload": f"tsi-hex8-linear-{n}^3 (strong-scaled over {world} GPU)",
           "baseline_config": "BASELINE.json configs[4] (monolithic TSI two-field tangent)",
           "value": m.n_ele_global / wall, "unit": "element-evaluations/s (two-field tangent)",
           "ms_per_step": 1e3 * wall, "elements_global": m.n_ele_global,
           "elements_evaluated_rank0": m.n_ele, "setup_s_rank0": t_setup,
           "path": "fused structured sweep (fcg_tsi_evaluate_fused)",
           "roofline": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": gbs / HBM_PEAK_GBS, "alg_bytes_rank0": byt,
                        "note": "algorithmic bytes: the four matrices and two residuals written "
                                "once, X / u / v / T read once per node (rank 0's share over the "
                                "max-over-ranks time)"},
           "cpu_baseline": None}
    for o in (tev, ev):
        o.close()
    if cpu_threads_ and rank == 0 and world == 1:
        try:
            out["cpu_baseline"] = tsi_cpu_baseline(n, 16, cpu_threads_)
        except Exception as e:  # report, never hide
            out["cpu_baseline"] = {"value": None, "error": repr(e)}
    return out


def _ctl_max(x, world):
    """Max over ranks of a host float (the control plane: gloo on the CPU)."""
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.item()


def _bcast_id(world):
    """rank 0's RCCL id to every rank over the gloo control plane."""
    def f(b):
        box = [b]
        if world > 1:
            dist.broadcast_object_list(box, src=0)
        return box[0]
    return f


def optionb_secondary(dev, rank, world, n, steps, staged):
    """SURVEY §8e option B, north_star's "RCCL all-reduce over xGMI of the shared-DOF residual":
    strict element partition (every rank only its GridGenerator box, no ghost layer; FCG_BOX_STRICT)
    -> set_state import of the interface displacements -> struct_calc_internalforce of the rank's
    elements into owned + extended rows -> fcg_shared_reduce (ncclAllReduce of the compact
    interface buffer, positions by (owner, GID)) -> the residual norm over the ranks."""
    comm = None
    try:
        iv = weak_interval(n, world)
        m = fcg.BoxMesh(fcg.HEX8, iv, upper=(iv[0] / n, iv[1] / n, iv[2] / n), jitter=0.1,
                        seed=20251015, rank=rank, nranks=world, strict=True)
        comm = None if staged else halo.Comm(rank, world, dev.index, _bcast_id(world))
        xchg = halo.gloo_exchange() if staged else comm.exchange
        n_own = m.n_owned_rows
        plan = halo.ImportPlan(rank, world, m.row_gid[:n_own], m.col_gid, halo.col_owner_of(m), xchg)
        h = halo.Halo(plan, dev.index)
        sp = halo.SharedPlan.of_mesh(m, xchg)
        sh = halo.Shared(sp, dev.index)
        ev = fcg.Evaluator(m, kinematics=fcg.LINEAR, youngs=210.0, poisson=0.3, device=dev.index)
        ev.set_async(True)
        u_h = m.u_col(1e-3)
        u_row = torch.from_numpy(np.ascontiguousarray(u_h[:n_own])).to(dev)  # row LID == col LID
        u_col = torch.zeros(m.n_cols, dtype=torch.float64, device=dev)
        f = torch.zeros(m.n_rows, dtype=torch.float64, device=dev)
        stream = torch.cuda.current_stream(dev)

        def step(marks=None):
            if staged:
                h.import_staged(u_row, u_col, stream)
            else:
                h.import_(comm, u_row, u_col, stream)
            ev.evaluate_device(fcg.CALC_INTERNALFORCE, fcg.OVERWRITE, u_col, f, stream=stream)
            if marks is not None:
                marks[0].record(stream)
            if staged:
                sh.reduce_staged(f, stream)
            else:
                sh.reduce(comm, f, stream)
            if marks is not None:
                marks[1].record(stream)
            if staged:
                loc = halo.residual_norm(f[:n_own], None, stream)
                t = torch.tensor([loc * loc], dtype=torch.float64)
                if world > 1:
                    dist.all_reduce(t)
                nrm = float(np.sqrt(t.item()))
            else:
                nrm = halo.residual_norm(f[:n_own], comm, stream)
            ev.check_error()
            return nrm

        for _ in range(5):
            step()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            nrm = step()
        torch.cuda.synchronize(dev)
        wall = _ctl_max((time.perf_counter() - t0) / steps, world)
        red = []
        for _ in range(3):
            mk = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            step(mk)
            red.append(mk[0].elapsed_time(mk[1]))
        ms_reduce = _ctl_max(float(np.mean(red)), world)
        out = {"workload": f"hex8-linear-{n}^3-per-gpu strict partition, internal force + shared-DOF "
                           f"all-reduce (option B)",
               "baseline_config": "BASELINE.json configs[3] (RCCL shared-DOF all-reduce)",
               "value": m.n_ele_global / wall, "unit": "element-evaluations/s (residual only)",
               "ms_per_step": 1e3 * wall, "elements_global": m.n_ele_global,
               "elements_evaluated_rank0": m.n_ele, "interface_dofs_global": sp.n_global,
               "allreduce_bytes": 8 * sp.n_global, "ms_shared_reduce_max": ms_reduce,
               "rccl_comm_size": comm.size() if comm is not None else None,
               "residual_norm": nrm,
               "transport": "host-staged gloo" if staged else "RCCL (fcg_halo_import + fcg_shared_reduce)"}
        for o in (sh, h, ev):
            o.close()
        return out
    except Exception as e:  # report, never hide
        return {"workload": "option-B shared-DOF all-reduce", "error": repr(e)}
    finally:
        if comm is not None:
            comm.close()


def host_secondary(dev, n, steps):
    """The 4C drop-in on host (Epetra-shaped) storage: fcg_evaluate_host with u, f and K in host
    memory, PCIe transfers included (pinned staging chunks, DMA overlapped with the host copy).
    OVERWRITE = the caller's SparseMatrix::zero() fused (K and f only written back); ACCUMULATE =
    fcg_evaluate's += (K and f also uploaded)."""
    try:
        mesh = fcg.BoxMesh(fcg.HEX8, (n, n, n), jitter=0.1, seed=20251015)
        ev = fcg.Evaluator(mesh, kinematics=fcg.LINEAR, youngs=210.0, poisson=0.3, device=dev.index)
        u = mesh.u_col(1e-3)
        K = np.zeros(mesh.nnz)
        f = np.zeros(mesh.n_rows)
        out = {"workload": f"hex8-linear-{n}^3 on host buffers (fcg_evaluate_host, PCIe-inclusive)",
               "baseline_config": "BASELINE.json configs[1] through the 4C host boundary",
               "unit": "element-evaluations/s", "K_bytes": 8 * mesh.nnz}
        for name, mode in (("overwrite", fcg.OVERWRITE), ("accumulate", fcg.ACCUMULATE)):
            ev.evaluate_host(fcg.CALC_NLNSTIFF, mode, u, f, K)  # first call: staging buffers
            t0 = time.perf_counter()
            for _ in range(steps):
                ev.evaluate_host(fcg.CALC_NLNSTIFF, mode, u, f, K)
            wall = (time.perf_counter() - t0) / steps
            out[name] = {"value": mesh.n_ele / wall, "ms_per_step": 1e3 * wall,
                         "pcie_gbs": (8 * mesh.nnz * (1 if mode == fcg.OVERWRITE else 2)) / wall / 1e9}
        out["value"] = out["overwrite"]["value"]
        ev.close()
        return out
    except Exception as e:  # report, never hide
        return {"workload": "host-buffer drop-in", "error": repr(e)}


def gather_secondary(dev, n, steps):
    """Config 2's element on an unstructured mesh: the n^3 hex8 box renumbered like an input-file
    mesh (random node and element numbering, no lattice hint: fcg.Discretization.renumbered) on
    the node-row gather path (FCG_PATH_GATHER, what any mesh without a lattice takes); linear and
    TotLag K + r, kernel time by hipEvents, HBM fraction by SURVEY §8d's bytes per element.  The
    "auto" entry: the same mesh under FCG_PATH_AUTO, where fcg_create finds the lattice in the
    connectivity and takes the row-block sweep."""
    try:
        box = fcg.BoxMesh(fcg.HEX8, (n, n, n), jitter=0.1, seed=20251015)
        dis = fcg.Discretization.renumbered(box, seed=1)
        del box
        out = {"workload": f"hex8-{n}^3 renumbered (unstructured: random node/element order)",
               "baseline_config": "BASELINE.json configs[1] element on a mesh without lattice",
               "unit": "element-evaluations/s", "elements": dis.n_ele, "nnz": dis.nnz}
        rng = np.random.default_rng(3)
        for name, kinem, amp, path in (("linear", fcg.LINEAR, 1e-3, fcg.PATH_GATHER),
                                       ("totlag", fcg.TOTLAG, 5e-2, fcg.PATH_GATHER),
                                       ("auto_linear", fcg.LINEAR, 1e-3, fcg.PATH_AUTO)):
            ev = fcg.Evaluator(dis, kinematics=kinem, youngs=210.0, poisson=0.3, device=dev.index,
                               path=path)
            u = torch.from_numpy(rng.standard_normal(dis.n_cols) * amp).to(dev)
            f = torch.zeros(dis.n_rows, dtype=torch.float64, device=dev)
            K = torch.zeros(dis.nnz, dtype=torch.float64, device=dev)
            for _ in range(3):
                ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, u, f, K)
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for _ in range(steps):
                ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, u, f, K)
            torch.cuda.synchronize(dev)
            wall = (time.perf_counter() - t0) / steps
            ev.set_timing(True)
            ts = []
            for _ in range(steps):
                ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, u, f, K)
                ts.append(sum(ev.timing()))
            ms_kern = float(np.mean(ts))
            gbs = ALG_BYTES_PER_ELE * dis.n_ele / (ms_kern * 1e-3) / 1e9
            out[name] = {"value": dis.n_ele / wall, "ms_per_step": 1e3 * wall, "ms_kernel": ms_kern,
                         "path": {fcg.PATH_GATHER: "gather", fcg.PATH_GENERAL: "general",
                                  fcg.PATH_STRUCTURED: "structured (lattice found in the connectivity)"}.get(
                             int(ev.info.path), int(ev.info.path)),
                         "roofline": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS,
                                      "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS}}
            ev.close()
            del K, f, u
            torch.cuda.empty_cache()
        out["value"] = out["linear"]["value"]
        return out
    except Exception as e:  # report, never hide
        return {"workload": "hex8 renumbered (gather path)", "error": repr(e)}


def totlag_sweep_secondary(dev, n, steps, with_pmc):
    """Config 2's mesh (n^3 hex8 GridGenerator box) with StVK total-Lagrangian kinematics
    (4C_solid_3D_ele_calc_displacement_based.hpp:45-72: F from the current coordinates, E, S, B_NL,
    K_geo) on the structured row-block sweep (sweep_h8_kernel<TotLag>): K + r per step, kernel time
    by hipEvents, HBM fraction by SURVEY §8d's bytes per element and the HBM traffic from counters
    of this run."""
    try:
        mesh = fcg.BoxMesh(fcg.HEX8, (n, n, n), jitter=0.1, seed=20251015)
        ev = fcg.Evaluator(mesh, kinematics=fcg.TOTLAG, youngs=210.0, poisson=0.3, device=dev.index)
        u = torch.from_numpy(mesh.u_col(5e-2)).to(dev)
        f = torch.zeros(mesh.n_rows, dtype=torch.float64, device=dev)
        K = torch.zeros(mesh.nnz, dtype=torch.float64, device=dev)
        for _ in range(5):
            ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, u, f, K)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(steps):
            ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, u, f, K)
        torch.cuda.synchronize(dev)
        wall = (time.perf_counter() - t0) / steps
        ev.set_timing(True)
        ts = []
        for _ in range(steps):
            ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, u, f, K)
            ts.append(sum(ev.timing()))
        ms_kern = float(np.mean(ts))
        alg = ALG_BYTES_PER_ELE * mesh.n_ele
        gbs = alg / (ms_kern * 1e-3) / 1e9
        path = int(ev.info.path)
        out = {"workload": f"hex8-totlag-{n}^3 structured (sweep)",
               "baseline_config": "BASELINE.json configs[1] mesh, StVK total Lagrangian",
               "value": mesh.n_ele / wall, "unit": "element-evaluations/s", "ms_per_step": 1e3 * wall,
               "ms_kernel": ms_kern, "elements": mesh.n_ele, "nnz": mesh.nnz,
               "path": "structured" if path == fcg.PATH_STRUCTURED else path,
               "roofline": {"bound": "hbm", "kernel": "sweep_h8_kernel<1,...> (TotLag)",
                            "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                            "frac": gbs / HBM_PEAK_GBS, "alg_bytes_per_element": ALG_BYTES_PER_ELE,
                            "alg_bytes_per_launch": alg}}
        ev.close()
        del K, f, u
        torch.cuda.empty_cache()
        if with_pmc:
            tr = measure_traffic(n, kernel="sweep_h8_kernel<1", extra=("--kinem", "totlag"))
            if "error" not in tr:
                tr["ratio_to_algorithmic"] = tr["hbm_bytes_per_evaluate"] / alg
                out["roofline"]["traffic"] = tr["hbm_bytes_per_evaluate"]
            out["roofline"]["traffic_detail"] = tr
        return out
    except Exception as e:  # report, never hide
        return {"workload": "hex8-totlag structured (sweep)", "error": repr(e)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--elems-per-dir", dest="n", type=int, default=100,
                    help="elements per direction per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baseline threads (0: the CPU share of this process)")
    ap.add_argument("--no-hex27", action="store_true", help="skip the hex27 (config 3) line")
    ap.add_argument("--no-tsi", action="store_true", help="skip the TSI (config 5) line")
    ap.add_argument("--hex27-n", type=int, default=40)
    ap.add_argument("--no-newton", action="store_true", help="skip the config-3 Newton line")
    ap.add_argument("--no-amg", action="store_true",
                    help="skip the unstructured-mesh Newton line (native AMG)")
    ap.add_argument("--newton-n", type=int, default=100)
    ap.add_argument("--no-totlag", action="store_true",
                    help="skip the structured hex8 TotLag sweep line")
    ap.add_argument("--no-slab", action="store_true",
                    help="skip the config-3 mesh under the slab schedule of the hex27 records")
    ap.add_argument("--no-optionb", action="store_true", help="skip the option-B (shared-DOF) line")
    ap.add_argument("--no-host", action="store_true", help="skip the host-buffer drop-in line")
    ap.add_argument("--timing-after", dest="timing_before", action="store_false",
                    help="no hipEvent pass before the warm-up (the kernel-duration pass after the "
                         "timed steps always runs)")
    ap.add_argument("--peaks-after", action="store_true",
                    help="measure the box's peaks after the timed steps instead of before the warm-up")
    ap.add_argument("--no-pmc", action="store_true",
                    help="no in-run rocprofv3 counter passes for roofline.traffic")
    ap.add_argument("--pmc-json", default=None,
                    help="committed PMC file to fall back on (default: newest profiles/pmc_rNN_vM.json)")
    ap.add_argument("--no-gather", action="store_true",
                    help="skip the unstructured (renumbered) hex8 line")
    ap.add_argument("--only-primary", action="store_true",
                    help="the primary line alone (no secondary lines, no CPU baseline, no counter "
                         "passes): the command whose rocprofv3 kernel statistics are committed")
    args = ap.parse_args()
    if args.only_primary:
        for k in ("no_cpu_baseline", "no_hex27", "no_tsi", "no_newton", "no_amg", "no_optionb",
                  "no_host", "no_pmc", "no_gather", "no_slab", "no_totlag"):
            setattr(args, k, True)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # data path: the library's RCCL communicator (halo import, norms); the control plane (RCCL id,
    # barriers, max over ranks) is gloo on the CPU.  FCG_DIST_BACKEND=gloo rehearses the multi-rank
    # flow with several ranks on one GPU (RCCL refuses that): halo staged through the host.
    staged = os.environ.get("FCG_DIST_BACKEND", "rccl") == "gloo"
    local = local % max(1, torch.cuda.device_count()) if staged else local
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    comm = None
    if world > 1:
        os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")
        dist.init_process_group("gloo")
        if not staged:
            comm = halo.Comm(rank, world, local, _bcast_id(world))

    iv = weak_interval(args.n, world)
    t_setup = time.perf_counter()
    mesh = fcg.BoxMesh(fcg.HEX8, iv, lower=(0.0, 0.0, 0.0),
                       upper=(iv[0] / args.n, iv[1] / args.n, iv[2] / args.n),
                       jitter=0.1, seed=20251015, rank=rank, nranks=world)
    ev = fcg.Evaluator(mesh, kinematics=fcg.LINEAR, youngs=210.0, poisson=0.3, device=local)
    t_setup = time.perf_counter() - t_setup

    u_col_h = mesh.u_col(1e-3)
    col_lid_of_row = {int(g): i for i, g in enumerate(mesh.col_gid)}
    u_row = torch.from_numpy(u_col_h[[col_lid_of_row[int(g)] for g in mesh.row_gid]]).to(dev)
    u_col = torch.zeros(mesh.n_cols, dtype=torch.float64, device=dev)
    f = torch.zeros(mesh.n_rows, dtype=torch.float64, device=dev)
    K = torch.zeros(mesh.nnz, dtype=torch.float64, device=dev)
    imp = None
    if world > 1:
        plan = halo.ImportPlan(rank, world, mesh.row_gid, mesh.col_gid, halo.col_owner_of(mesh),
                               halo.gloo_exchange() if staged else comm.exchange)
        imp = halo.Halo(plan, local)
    else:
        u_col.copy_(torch.from_numpy(u_col_h).to(dev))
    stream = torch.cuda.current_stream(dev)
    # evaluate returns once queued; 4C's throws are collected after the norm (one drain per step)
    ev.set_async(True)

    def step(marks=None, norm=True):
        if marks is not None:
            marks[0].record(stream)
        if imp is not None:
            if staged:
                imp.import_staged(u_row, u_col, stream)
            else:
                imp.import_(comm, u_row, u_col, stream)
        if marks is not None:
            marks[1].record(stream)
        ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, u_col, f, K, stream=stream)
        if marks is not None:
            marks[2].record(stream)
            marks[2].synchronize()
            marks.append(time.perf_counter())
        if not norm:
            return None
        if staged and world > 1:
            loc = halo.residual_norm(f, None, stream)
            t = torch.tensor([loc * loc], dtype=torch.float64)
            dist.all_reduce(t)
            nrm = float(np.sqrt(t.item()))
        else:
            nrm = halo.residual_norm(f, comm, stream)
        if marks is not None:
            marks.append(time.perf_counter())
        ev.check_error()
        return nrm

    def phase_pass(n):
        """Where a step's time goes on this rank (a separate pass, outside the timed window):
        set_state import (halo) and evaluate by hipEvents on the launch stream, the residual norm
        (sum of squares + RCCL all-reduce + read-back, blocking) by the host clock."""
        halo_ms, eval_ms, norm_ms = [], [], []
        for _ in range(n):
            mk = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            step(mk)
            halo_ms.append(mk[0].elapsed_time(mk[1]))
            eval_ms.append(mk[1].elapsed_time(mk[2]))
            norm_ms.append(1e3 * (mk[4] - mk[3]))
        return {"ms_halo_import": float(np.mean(halo_ms)), "ms_evaluate": float(np.mean(eval_ms)),
                "ms_norm_allreduce": float(np.mean(norm_ms))}

    # SURVEY §8d asks for the spec peaks re-measured on the box; measured here, on every rank's
    # GPU before its warm-up, so that the timed steps start on a GPU already at its working
    # clocks (the reported peaks are rank 0's)
    peaks = None
    if not args.peaks_after:
        try:
            peaks = fcg.measure_peaks(dev.index) + fcg.measure_hbm(dev.index)
        except Exception as e:  # report, never hide
            peaks = e
    # the kernel's own duration (hipEvents on its launch stream) from a separate pass of K steps,
    # so that the event records and queries stay out of the wall-clock window; run before the
    # warm-up by default (--timing-after: after the timed steps)
    def kernel_timing_pass():
        ev.set_timing(True)
        t_e, t_a = [], []
        for _ in range(args.steps):
            step()
            a, b = ev.timing()
            t_e.append(a)
            t_a.append(b)
        torch.cuda.synchronize(dev)
        ev.set_timing(False)
        return t_e, t_a

    # a first hipEvent pass before the warm-up also brings the GPU from its idle clocks to its
    # working clocks (measured: with 5 warm-up steps alone the 20 timed steps average 1.07 ms,
    # with this pass in front 1.03 ms, at an unchanged warm kernel time); its kernel times are
    # reported as ms_kernel_cold, the roofline uses the pass after the timed steps
    cold = kernel_timing_pass() if args.timing_before else None
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    # the timed steps: set_state import (N > 1) + evaluate, queued back to back; the element-error
    # flags (sticky across the queued evaluates) are read once after the K steps, inside the
    # window.  The residual norm is a Newton-loop ingredient outside the assembly path: computed
    # after the window and timed per step in the rank phases (ms_norm_allreduce).
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(norm=False)
    ev.check_error()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    nrm = step()
    t_el, t_as = kernel_timing_pass()
    phases = phase_pass(max(3, min(args.steps, 10)))
    rank_info = dict(rank=rank, device=local, elements_owned=int(mesh.n_ele_row),
                     elements_ghost=int(mesh.n_ele - mesh.n_ele_row),
                     elements_evaluated=int(mesh.n_ele), dofs_owned=int(mesh.n_rows),
                     nnz=int(mesh.nnz),
                     halo_send_doubles=imp.n_send if imp is not None else 0,
                     halo_recv_doubles=imp.n_recv if imp is not None else 0,
                     halo_bytes=8 * ((imp.n_send + imp.n_recv) if imp is not None else 0),
                     ms_kernel=float(np.mean(t_el) + np.mean(t_as)), **phases)
    ranks = [None] * world
    if world > 1:
        dist.all_gather_object(ranks, rank_info)
    else:
        ranks = [rank_info]
    if peaks is None:
        try:
            peaks = fcg.measure_peaks(dev.index) + fcg.measure_hbm(dev.index)
        except Exception as e:  # report, never hide
            peaks = e
    elapsed = _ctl_max(t1 - t0, world)
    ms_step = 1e3 * elapsed / args.steps
    n_ele_global = mesh.n_ele_global
    value = n_ele_global / (elapsed / args.steps)

    ms_el = float(np.mean(t_el))
    ms_as = float(np.mean(t_as))
    ms_kern = ms_el + ms_as
    n_row_ele = mesh.n_ele_row
    achieved = ALG_BYTES_PER_ELE * n_row_ele / (ms_kern * 1e-3) / 1e9
    flops = ALG_FLOP_PER_ELE * n_row_ele / (ms_kern * 1e-3) / 1e12
    traffic, traffic_source, traffic_detail = None, None, None
    if rank == 0 and world == 1 and not args.no_pmc and ev.info.path == fcg.PATH_STRUCTURED:
        traffic_detail = measure_traffic(args.n)
        if "error" not in traffic_detail:
            traffic = traffic_detail["hbm_bytes_per_evaluate"]
            traffic_source = "this run (rocprofv3 --pmc, child passes)"
    if traffic is None:
        # fall back to a committed PMC pass of this kernel (tools/pmc.sh + tools/pmc_traffic.py),
        # named in the output: it is not a measurement of this run
        pmc_path = committed_pmc(args.pmc_json)
        if pmc_path and os.path.exists(pmc_path):
            try:
                pmc = json.load(open(pmc_path))
                if pmc.get("workload") == f"hex8-linear-{args.n}^3-per-gpu":
                    traffic = pmc.get("hbm_bytes_per_evaluate")
                    traffic_source = (f"committed file profiles/{os.path.basename(pmc_path)} "
                                      f"(not measured in this run)")
            except Exception:
                traffic = None

    out = {
        "metric": "element-evaluations/sec (hex8 linear elasticity, K+r global assembly)",
        "value": value,
        "unit": "element-evaluations/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (GridGenerator box, jitter 0.1h, analytic displacement field)",
        "config": {
            "workload": f"hex8-linear-{args.n}^3-per-gpu",
            "baseline_config": "BASELINE.json configs[1] (1M hex8, K and r on 1 MI355X)"
                               if world == 1 else "BASELINE.json configs[3] (weak-scaled, RCCL)",
            "global_intervals": list(iv),
            "elements_global": n_ele_global,
            "elements_evaluated_per_gpu": mesh.n_ele,
            "dofs_owned_rank0": mesh.n_rows,
            "nnz_rank0": mesh.nnz,
            "material": "StVenantKirchhoff E=210 nu=0.3",
            "assembly": "zero+assemble fused (FCG_OVERWRITE), owned rows, no atomics",
            "step": ("set_state import (N > 1) + one evaluate (K and r), queued back to back; "
                     "element-error flags read once after the timed steps; residual norm outside "
                     "the window (rank phases: ms_norm_allreduce)"),
            "parallelism": (f"element partition x{world} (GridGenerator box split, ghost layer; "
                            f"set_state import by fcg_halo_import = RCCL grouped send/recv, "
                            f"residual norm after the timed steps by fcg_norm2 = RCCL all-reduce)" if not staged else
                            f"element partition x{world}, host-staged gloo rehearsal")
                           if world > 1 else "single GPU",
            "setup_s_rank0": t_setup,
        },
        # The bounding roofline of the launch: SURVEY.md §8d prices the K + r assembly FP64-bound
        # (41.4 kflop vs 2,069 B per hex8 element), but the kernel runs the isotropic (lambda, mu)
        # contraction, a fraction of those flops, on the VALU (no MFMA), and its floor in practice
        # is writing K once: so the reported bound is HBM (algorithmic bytes / kernel time vs the
        # 8 TB/s spec), and the FP64 fraction by SURVEY's flop count is kept beside it.
        "roofline": {
            "bound": "hbm",
            "kernel": ("sweep_h8_kernel (structured row-block sweep, one evaluate)"
                       if ev.info.path == fcg.PATH_STRUCTURED
                       else "element_kernel + assemble_kernel (one evaluate)"),
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "traffic_source": traffic_source,
            "traffic_detail": traffic_detail,
            "traffic_ratio_to_algorithmic": (traffic / (ALG_BYTES_PER_ELE * n_row_ele)
                                             if traffic else None),
            "alg_bytes_per_element": ALG_BYTES_PER_ELE,
            "elements_per_launch": n_row_ele,
            "ms_element_kernel": ms_el,
            "ms_assemble_kernel": ms_as,
            "ms_kernel_cold": float(np.mean(cold[0]) + np.mean(cold[1])) if cold else None,
            "fp64_valu": {"achieved_tflops_by_survey_count": flops, "peak_tflops": FP64_PEAK_TFS,
                          "frac": flops / FP64_PEAK_TFS, "alg_flop_per_element": ALG_FLOP_PER_ELE,
                          "note": "SURVEY §8d flop count; the isotropic contraction executes fewer"},
        },
        # one line per rank: its GridGenerator share, halo volume and where its step time went
        "ranks": ranks,
        "collectives": {
            "transport": ("RCCL (fcg_comm: grouped ncclSend/ncclRecv + ncclAllReduce)" if comm is not None
                          else "host-staged gloo" if world > 1 else "none (single GPU)"),
            "rccl_comm_size": comm.size() if comm is not None else None,
            "halo_bytes_per_step_total": int(sum(r["halo_bytes"] for r in ranks)) // 2,
            "norm_allreduce_bytes": 8 if world > 1 else 0,
            "ms_halo_import_max": max(r["ms_halo_import"] for r in ranks),
            "ms_norm_allreduce_max": max(r["ms_norm_allreduce"] for r in ranks),
            "note": "K and r need no exchange (ghost layer, owned rows; SURVEY §8e option A); "
                    "option B's interface all-reduce is the `optionb` secondary line",
        },
        "assembly_wall_ms": ms_step,
        # the round-1/2 step definition (norm all-reduce + flag read in every step), for comparison
        "ms_per_step_with_norm": ms_step + max(r["ms_norm_allreduce"] for r in ranks),
        "untimed_steps_before_timed": args.warmup + (args.steps if cold else 0),
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline(args.n, fcg.LINEAR, cpu_threads(args.cpu_threads))
        except Exception as e:  # report, never hide
            out["cpu_baseline"] = {"value": None, "error": repr(e)}
    # the spec peaks re-measured on this box (STREAM triad, FP64 VALU, FP64 MFMA);
    # `peak` stays the spec figure, the fractions against the measured ones are reported beside
    if rank == 0:
        try:
            if isinstance(peaks, Exception):
                raise peaks
            triad, valu, mfma, copy, write = peaks
            fp64_meas = max(valu, mfma)
            hbm_best = max(triad, copy, write)
            out["roofline"]["measured_peaks"] = {
                "hbm_triad_gbs": triad, "hbm_copy_gbs": copy, "hbm_write_only_gbs": write,
                "fp64_valu_tflops": valu, "fp64_mfma_tflops": mfma,
                "hbm_frac_vs_triad": achieved / triad if triad > 0 else None,
                "hbm_frac_vs_best_measured": achieved / hbm_best if hbm_best > 0 else None,
                "fp64_frac_vs_measured": flops / fp64_meas if fp64_meas > 0 else None}
        except Exception as e:  # report, never hide
            out["roofline"]["measured_peaks"] = {"error": repr(e)}
    out["residual_norm"] = nrm
    # the other BASELINE configs' kernels, measured after the primary line's buffers are freed
    if imp is not None:
        imp.close()
    del K, f, u_col, u_row, imp
    ev.close()
    torch.cuda.empty_cache()
    secondary = []
    if not args.no_optionb:
        secondary.append(optionb_secondary(dev, rank, world, args.n, max(3, min(args.steps, 10)),
                                           staged))
        torch.cuda.empty_cache()
    if not args.no_tsi:
        secondary.append(tsi_secondary(dev, rank, world, max(3, min(args.steps, 10)),
                                       cpu_threads_=0 if args.no_cpu_baseline
                                       else cpu_threads(args.cpu_threads)))
    if rank == 0 and world == 1 and not args.no_host:
        secondary.append(host_secondary(dev, args.n, 3))
    if rank == 0 and world == 1 and not args.no_gather:
        secondary.append(gather_secondary(dev, args.n, max(3, min(args.steps, 10))))
    if rank == 0 and world == 1 and not args.no_totlag:
        secondary.append(totlag_sweep_secondary(dev, args.n, max(3, min(args.steps, 10)),
                                                not args.no_pmc))
        torch.cuda.empty_cache()
    if rank == 0 and world == 1 and not args.no_hex27:
        try:
            secondary.append(hex27_secondary(dev, args.hex27_n, max(3, min(args.steps, 10)),
                                             cpu_threads(args.cpu_threads), not args.no_cpu_baseline))
        except Exception as e:  # report, never hide
            secondary.append({"workload": "hex27-totlag", "error": repr(e)})
    if rank == 0 and world == 1 and not args.no_slab:
        torch.cuda.empty_cache()
        try:
            secondary.append(hex27_slab_secondary(dev, args.newton_n, 3, 5000))
        except Exception as e:  # report, never hide
            secondary.append({"workload": "hex27-slab-schedule", "error": repr(e)})
        torch.cuda.empty_cache()
    if rank == 0 and world == 1 and not args.no_newton:
        torch.cuda.empty_cache()
        try:
            h27cpu = next((x.get("cpu_baseline") for x in secondary
                           if str(x.get("workload", "")).startswith("hex27-totlag-") and
                           isinstance(x.get("cpu_baseline"), dict) and x["cpu_baseline"].get("value")), None)
            secondary.append(newton_secondary(args.newton_n, cpu_rate=h27cpu))
        except Exception as e:  # report, never hide
            secondary.append({"workload": "hex27-totlag-newton", "error": repr(e)})
    if rank == 0 and world == 1 and not args.no_amg:
        torch.cuda.empty_cache()
        try:
            secondary.append(amg_newton_secondary(args.n))
        except Exception as e:  # report, never hide
            secondary.append({"workload": "hex8-renumbered-newton-amg", "error": repr(e)})
    # the hex27 element's MFMA rate against this box's measured FP64 MFMA peak as well
    if not isinstance(peaks, Exception) and peaks is not None:
        for sec in secondary:
            mf = sec.get("roofline", {}).get("mfma_counters") if isinstance(sec, dict) else None
            if mf and "mfma_tflops" in mf and peaks[2] > 0:
                mf["measured_mfma_peak_tflops"] = peaks[2]
                mf["mfma_frac_of_measured_peak"] = mf["mfma_tflops"] / peaks[2]
    if secondary:
        out["secondary"] = secondary
    if rank == 0:
        print(json.dumps(out))
    if comm is not None:
        comm.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
