"""Newton-loop measurement on one GPU (BASELINE configs 1 and 3 shapes).

Cantilever box [0,L]x[0,1]x[0,1] (x- face clamped, x+ face surface load), StVK E=210 nu=0.3,
static full Newton through 4c_amd/newton.py: per iteration fcg_evaluate_device + Dirichlet +
block-Jacobi PCG.  Prints one JSON line with per-phase times.
usage: newton_bench.py --celltype hex8|hex27 --kinem linear|totlag --n N [--load L]"""
import argparse
import importlib
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
pkg = importlib.import_module("4c_amd")
fcg, newton = pkg.fcg, importlib.import_module("4c_amd.newton")

ap = argparse.ArgumentParser()
ap.add_argument("--celltype", default="hex8")
ap.add_argument("--kinem", default="linear")
ap.add_argument("--n", type=int, default=10)
ap.add_argument("--length", type=float, default=10.0)
ap.add_argument("--load", type=float, default=-1e-3)
ap.add_argument("--lin-rtol", type=float, default=1e-10)
ap.add_argument("--tol", type=float, default=1e-8)
ap.add_argument("--path", default="auto", choices=["auto", "general", "structured"])
ap.add_argument("--lin-max-iter", type=int, default=100000)
ap.add_argument("--forcing", default="Constant", choices=["Constant", "Type 1", "Type 2"],
                help="NOX forcing-term method (Constant = --lin-rtol every step)")
ap.add_argument("--mg", action="store_true",
                help="geometric multigrid preconditioned flexible CG (4c_amd/multigrid.py)")
ap.add_argument("--mg-nu", type=int, default=2, help="Chebyshev degree of the MG smoother")
ap.add_argument("--mg-coarse-rtol", type=float, default=1e-2)
ap.add_argument("--mg-ratio", type=float, default=None,
                help="Chebyshev eigenvalue ratio (default: the solver's own)")
ap.add_argument("--mg-mixed", action="store_true", help="FP32 copy of K in the fine smoother")
ap.add_argument("--mg-no-fine-post", action="store_true",
                help="no post-smoothing on the finest level (pre-smoothing V-cycle there)")
ap.add_argument("--mg-matrix-free", action="store_true",
                help="hex27: the fine level's smoother and V-cycle residual apply K(u) element by "
                     "element (fcg_tangent_apply) instead of reading the assembled K")
ap.add_argument("--mg-outer-matrix-free", action="store_true",
                help="with --mg-matrix-free: the outer flexible CG applies the same tangent "
                     "element by element too (the assembled K still sets the smoother's blocks)")
ap.add_argument("--mg-coarse", default="auto", choices=["auto", "dense", "pcg", "amg"],
                help="coarsest-level solver of the geometric multigrid")
ap.add_argument("--amg", action="store_true",
                help="smoothed-aggregation AMG preconditioned flexible CG (4c_amd/amg.py)")
ap.add_argument("--amg-native", action="store_true",
                help="the same AMG as the native C-ABI object (fcg_amg_create / fcg_amg_solve)")
ap.add_argument("--renumber", action="store_true",
                help="solve on the box renumbered as an input-file mesh (no lattice, random order)")
a = ap.parse_args()
ct = fcg.HEX8 if a.celltype == "hex8" else fcg.HEX27
kin = fcg.LINEAR if a.kinem == "linear" else fcg.TOTLAG
t0 = time.perf_counter()
mesh = fcg.BoxMesh(ct, (a.n, a.n, a.n), upper=(a.length, 1.0, 1.0))
X = mesh.node_x
dbc_nodes = np.nonzero(np.isclose(X[:, 0], 0.0) & (mesh.node_dof_row >= 0))[0]
dbc = np.sort((mesh.node_dof_row[dbc_nodes][:, None] + np.arange(3)).ravel()).astype(np.int32)
face = [1, 2, 6, 5] if ct == fcg.HEX8 else [1, 2, 6, 5, 9, 14, 17, 13, 22]
faces = mesh.ele_nodes[mesh.ele_ijk[:, 0] == a.n - 1][:, face]
fext = np.zeros(mesh.n_rows)
fcg.neumann_surface(ct, faces, X, mesh.node_dof_row, [1, 1, 1], [0.0, 0.0, a.load], fext)
path = {"auto": fcg.PATH_AUTO, "general": fcg.PATH_GENERAL, "structured": fcg.PATH_STRUCTURED}[a.path]
box = mesh
if a.renumber:
    mesh = fcg.Discretization.renumbered(box, seed=1)
    newrow = (3 * mesh.node_perm[:, None] + np.arange(3)).ravel()  # box rows are 3 * node + d
    f2 = np.zeros_like(fext)
    f2[newrow] = fext
    fext = f2
    dbc = np.sort(newrow[dbc]).astype(np.int32)
t_mesh = time.perf_counter() - t0
print(f"mesh {t_mesh:.1f} s: {mesh.n_ele} elements, {mesh.nnz} nonzeros", file=sys.stderr, flush=True)
ev = fcg.Evaluator(mesh, kinematics=kin, youngs=210.0, poisson=0.3, path=path)
t_setup = time.perf_counter() - t0
setup_phases = {"mesh_s": t_mesh, "create_s": t_setup - t_mesh,
                "create_phases_s": ev.create_phases()}
print(f"fcg_create {t_setup - t_mesh:.1f} s: {json.dumps(setup_phases['create_phases_s'])}", file=sys.stderr, flush=True)


class Timed(newton.StaticNewton):
    """StaticNewton with per-phase timing (synchronised wall clock)."""

    def solve(self):
        u = torch.zeros(self.n, dtype=torch.float64, device=self.dev)
        self.history, ndu = [], float("inf")
        nr_old = lin_abs = None
        for it in range(self.max_iter + 1):
            torch.cuda.synchronize()
            t_a = time.perf_counter()
            self.ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, u, self.fint, self.K)
            torch.cuda.synchronize()
            t_b = time.perf_counter()
            torch.sub(self.fint, self.fext, out=self.r)
            self.ev.dirichlet_apply(self.dbc, self.K, self.r, self.freact)
            nr = float(torch.linalg.vector_norm(self.r))
            t_c = time.perf_counter()
            rec = {"iter": it, "norm_res": nr, "assembly_ms": 1e3 * (t_b - t_a),
                   "dbc_ms": 1e3 * (t_c - t_b)}
            if it > 0 and nr <= self.tol_res and ndu <= self.tol_inc:
                self.history.append(rec)
                return u
            torch.neg(self.r, out=self.r)
            # heartbeat while the (blocking) PCG runs: the GPU box treats 3 silent minutes as a hang
            import threading
            done = threading.Event()
            hb = threading.Thread(target=lambda: [print(f"  pcg running ({it})", file=sys.stderr,
                                                        flush=True) for _ in iter(lambda: done.wait(30), True)])
            hb.start()
            try:
                eta = self.forcing.compute(it, nr, nr_old, lin_abs)
                if hasattr(self.linear_solver, "set_state"):
                    self.linear_solver.set_state(u)
                li, lr = self.linear_solve(self.r, self.du, eta)
                nr_old, lin_abs = nr, lr * nr
            finally:
                done.set()
                hb.join()
            torch.cuda.synchronize()
            t_d = time.perf_counter()
            ndu = float(torch.linalg.vector_norm(self.du))
            u += self.du
            rec.update(solve_ms=1e3 * (t_d - t_c), pcg_iter=li, pcg_relres=lr, eta=eta, norm_inc=ndu)
            self.history.append(rec)
            print(json.dumps(rec), file=sys.stderr, flush=True)
        # as StaticNewton: an unconverged loop is an error, never a timing
        raise RuntimeError(f"Newton did not converge in {self.max_iter} iterations: "
                           f"{self.history[-3:]}")


mg = None
if a.mg:
    t_mg = time.perf_counter()
    mg = importlib.import_module("4c_amd.multigrid").Multigrid(
        mesh, ev, lambda m: np.isclose(m.node_x[:, 0], 0.0), 210.0, 0.3, nu=a.mg_nu,
        coarse_rtol=a.mg_coarse_rtol, mixed=a.mg_mixed, coarse_solver=a.mg_coarse,
        fine_post=not a.mg_no_fine_post, matrix_free=a.mg_matrix_free,
        outer_matrix_free=a.mg_outer_matrix_free,
        **({"ratio": a.mg_ratio} if a.mg_ratio else {}))
    setup_phases["multigrid_s"] = time.perf_counter() - t_mg
    print(f"multigrid setup {time.perf_counter() - t_mg:.1f} s: {json.dumps(mg.describe())}",
          file=sys.stderr, flush=True)
    t_setup = time.perf_counter() - t0
if a.amg or a.amg_native:
    t_mg = time.perf_counter()
    amg_mod = importlib.import_module("4c_amd.amg")
    kw = {"ratio": a.mg_ratio} if a.mg_ratio else {}
    mg = (amg_mod.NativeAMG(mesh, ev, dbc, nu=a.mg_nu, **kw) if a.amg_native
          else amg_mod.AMG(mesh, ev, dbc, nu=a.mg_nu, **kw))
    t_amg_setup = time.perf_counter() - t_mg
    setup_phases["amg_s"] = t_amg_setup
    print(f"AMG setup (host graph) {t_amg_setup:.1f} s: {json.dumps(mg.describe())}",
          file=sys.stderr, flush=True)
    t_setup = time.perf_counter() - t0
nt = Timed(ev, fext, dbc, lin_max_iter=a.lin_max_iter, tol_res=a.tol * max(np.linalg.norm(fext), 1e-300), tol_inc=a.tol,
           lin_rtol=a.lin_rtol, max_iter=40,
           forcing=newton.ForcingTerm(a.forcing, constant=a.lin_rtol), linear_solver=mg)
# the kernels of the Newton step launched once on scratch data (setup: HIP loads a kernel's code
# object at its first launch, ~0.3 s of config 3's first Newton step otherwise)
t_w = time.perf_counter()
if hasattr(mg, "warm_up"):
    mg.warm_up()
nt.warm_up()
setup_phases["warm_up_s"] = time.perf_counter() - t_w
t_setup = time.perf_counter() - t0
print(f"setup {t_setup:.1f} s (warm-up {setup_phases['warm_up_s']:.2f} s)", file=sys.stderr, flush=True)
t1 = time.perf_counter()
u = nt.solve()
torch.cuda.synchronize()
t_newton = time.perf_counter() - t1
h = nt.history
# the tangent at the solution (before Dirichlet rows) is symmetric for StVK: x.(K y) == y.(K x)
ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, u, nt.fint, nt.K)
gen = torch.Generator(device="cpu").manual_seed(7)
xv = torch.randn(mesh.n_rows, generator=gen, dtype=torch.float64).to(u.device)
yv = torch.randn(mesh.n_rows, generator=gen, dtype=torch.float64).to(u.device)
Kx, Ky = torch.empty_like(xv), torch.empty_like(yv)
ev.spmv(nt.K, xv, Kx)
ev.spmv(nt.K, yv, Ky)
sym = abs(float(torch.dot(xv, Ky)) - float(torch.dot(yv, Kx))) / float(
    torch.linalg.vector_norm(xv) * torch.linalg.vector_norm(Ky))
r_final = float(torch.linalg.vector_norm(nt.fint - nt.fext)) / max(np.linalg.norm(fext), 1e-300)
# the matrix-free tangent action the multigrid's smoother and outer FCG apply (hex27 StVK):
# its device time per application at the solution, hipEvents over 20 back-to-back applications
apply_ms = None
if a.mg and a.mg_matrix_free:
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev.tangent_apply(u, xv, Kx)
    e0.record()
    for _ in range(20):
        ev.tangent_apply(u, xv, Kx)
    e1.record()
    torch.cuda.synchronize()
    apply_ms = e0.elapsed_time(e1) / 20
del xv, yv, Kx, Ky
out = {"config": f"{a.celltype}-{a.kinem}-{a.n}^3-cantilever", "forcing": a.forcing,
       "converged": True, "tangent_symmetry_rel": sym,
       "residual_rel_incl_dbc_rows": r_final,
       "linear_solver": (f"multigrid-FCG (Chebyshev {a.mg_nu}"
                         + (", matrix-free fine smoother and outer operator)" if a.mg_outer_matrix_free else
                            ", matrix-free fine smoother)" if a.mg_matrix_free else ")") if a.mg else
                         f"SA-AMG-FCG (Chebyshev {a.mg_nu})" if a.amg else
                         f"SA-AMG-FCG native C ABI (Chebyshev {a.mg_nu})" if a.amg_native else
                         "block-Jacobi PCG"),
       "mesh": "renumbered (input-file order, no lattice)" if a.renumber else "GridGenerator box",
       "mg_levels": mg.describe() if mg else None, "elements": mesh.n_ele,
       "dofs": mesh.n_rows, "nnz": mesh.nnz, "h27_slabs": int(ev.info.h27_slabs),
       "scratch_bytes": int(ev.info.scratch_bytes), "setup_s": t_setup, "setup_phases": setup_phases, "newton_s": t_newton,
       "newton_iterations": len(h) - 1,
       "assembly_ms_mean": float(np.mean([r["assembly_ms"] for r in h])),
       "assembly_elem_per_s": mesh.n_ele / (1e-3 * float(np.median([r["assembly_ms"] for r in h]))),
       "solve_ms_total": float(sum(r.get("solve_ms", 0.0) for r in h)),
       "assembly_ms": [r["assembly_ms"] for r in h], "tangent_apply_ms": apply_ms,
       "pcg_iterations": [r.get("pcg_iter") for r in h[:-1]],
       "tip_uz": float(u[mesh.node_dof_row[np.argmax(mesh.node_x.sum(axis=1))] + 2]),
       "amg_graph_setup_s": t_amg_setup if (a.amg or a.amg_native) else None,
       "amg_numeric_setup_ms": mg.setup_ms if (a.amg or a.amg_native) else None,
       "amg_stats": mg.stats() if a.amg_native else None,
       "history": h}
print(json.dumps(out))
