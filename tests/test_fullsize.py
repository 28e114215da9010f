"""Parity at the sizes the bench runs (BASELINE configs 2/3 element shapes), beyond the small-mesh
parity of test_gpu_parity.py:

* hex8 StVK TotLag 100^3 (1M elements) and hex27 StVK TotLag 40^3 (64k elements, 298M nonzeros):
  the whole K and f_int against the oracle run with 16 workers as ranks (reference MPI
  semantics), at the tolerances of SURVEY §8d;
* the config-3 Newton loop (hex27 StVK TotLag cantilever, multigrid-preconditioned solve): the
  converged displacement is in equilibrium by the ORACLE's element forces on a sample of free
  nodes (an independent check of the converged solution, not of the library against itself),
  and the StVK TotLag tangent at the solution is symmetric (x.K y == y.K x through fcg_spmv).
  FCG_FULLSIZE_N (default 40) sets the cube size; 100 is config 3 itself (1M hex27).
"""

import importlib
import os

import numpy as np
import pytest

from parity_util import oracle_evaluate, rel_err

fcg = importlib.import_module("4c_amd").fcg
newton = importlib.import_module("4c_amd.newton")
torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu
E, NU = 210.0, 0.3


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


@pytest.mark.parametrize("celltype,n,amp", [(fcg.HEX8, 100, 5e-2), (fcg.HEX27, 40, 5e-2)])
def test_totlag_full_size_against_oracle(celltype, n, amp):
    dev = _dev()
    mesh = fcg.BoxMesh(celltype, (n, n, n), jitter=0.1 if celltype == fcg.HEX8 else 0.02,
                       seed=20251015)
    u = mesh.u_col(amp)
    ev = fcg.Evaluator(mesh, kinematics=fcg.TOTLAG, youngs=E, poisson=NU)
    f = torch.zeros(mesh.n_rows, dtype=torch.float64, device=dev)
    K = torch.full((mesh.nnz,), float("nan"), dtype=torch.float64, device=dev)
    ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, torch.from_numpy(u).to(dev), f, K)
    Kg, fg = K.cpu().numpy(), f.cpu().numpy()
    del K, f
    ev.close()
    err, _, Kr, fr = oracle_evaluate(mesh, fcg.TOTLAG, E, NU, u, nworkers=16)
    assert err == 0
    assert rel_err(fg, fr) <= 1e-10, rel_err(fg, fr)
    assert np.all(np.isfinite(Kg))
    assert rel_err(Kg, Kr) <= 1e-12, rel_err(Kg, Kr)
    assert np.abs(Kg - Kr).max() <= 1e-12 * np.abs(Kr).max()


# the bench's config-3 line (tools/newton_bench.py --celltype hex27 --kinem totlag --n 100 --mg,
# profiles/r01_config3_hex27_1M_totlag_newton_mg.json): tip displacement u_z at (1, 1, 1)
CONFIG3_TIP_UZ = -0.03406788471634048


@pytest.mark.parametrize("n", [int(os.environ.get("FCG_FULLSIZE_N", "40")), 100])
def test_config3_newton_equilibrium_and_symmetry(n):
    """n = 100 is BASELINE config 3 itself (1M hex27, 4.63e9 nonzeros)."""
    import oracle_lib as orc
    dev = _dev()
    mg_mod = importlib.import_module("4c_amd.multigrid")
    mesh = fcg.BoxMesh(fcg.HEX27, (n, n, n), upper=(1.0, 1.0, 1.0))
    X = mesh.node_x
    clamped = np.isclose(X[:, 0], 0.0)
    dbc_nodes = np.nonzero(clamped & (mesh.node_dof_row >= 0))[0]
    dbc = np.sort((mesh.node_dof_row[dbc_nodes][:, None] + np.arange(3)).ravel()).astype(np.int32)
    faces = mesh.ele_nodes[mesh.ele_ijk[:, 0] == n - 1][:, [1, 2, 6, 5, 9, 14, 17, 13, 22]]
    fext = np.zeros(mesh.n_rows)
    fcg.neumann_surface(fcg.HEX27, faces, X, mesh.node_dof_row, [1, 1, 1], [0.0, 0.0, -1.0], fext)
    ev = fcg.Evaluator(mesh, kinematics=fcg.TOTLAG, youngs=E, poisson=NU)
    mg = mg_mod.Multigrid(mesh, ev, lambda m: np.isclose(m.node_x[:, 0], 0.0), E, NU)
    nt = newton.StaticNewton(ev, fext, dbc, tol_res=1e-10 * np.linalg.norm(fext), tol_inc=1e-10,
                             max_iter=30, linear_solver=mg)
    u = nt.solve()
    assert nt.history[-1]["norm_res"] <= 1e-10 * np.linalg.norm(fext), nt.history
    uh = u.cpu().numpy()
    if n == 100:  # pins the bench's 1M Newton result
        tip = uh[mesh.node_dof_row[np.argmax(X.sum(axis=1))] + 2]
        assert abs(tip - CONFIG3_TIP_UZ) <= 1e-9 * abs(CONFIG3_TIP_UZ), tip
        assert len(nt.history) - 1 <= 6, nt.history
    # symmetry of the tangent at the solution (before Dirichlet rows): x.(K y) == y.(K x)
    K = torch.empty(mesh.nnz, dtype=torch.float64, device=dev)
    f = torch.empty(mesh.n_rows, dtype=torch.float64, device=dev)
    ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, u, f, K)
    g = torch.Generator(device="cpu").manual_seed(7)
    x = torch.randn(mesh.n_rows, generator=g, dtype=torch.float64).to(dev)
    y = torch.randn(mesh.n_rows, generator=g, dtype=torch.float64).to(dev)
    Kx, Ky = torch.empty_like(x), torch.empty_like(y)
    ev.spmv(K, x, Kx)
    ev.spmv(K, y, Ky)
    a, b = float(torch.dot(x, Ky)), float(torch.dot(y, Kx))
    scale = float(torch.linalg.vector_norm(x) * torch.linalg.vector_norm(Ky))
    assert abs(a - b) <= 1e-12 * scale, (a, b, scale)
    fint_lib = f.cpu().numpy()
    del K, Kx, Ky, x, y, f
    mg = nt = None
    ev.close()
    # equilibrium by the oracle's element forces at 300 sampled free nodes
    rng = np.random.default_rng(11)
    own = np.nonzero((mesh.node_dof_row >= 0) & ~clamped)[0]
    sample = rng.choice(own, size=min(300, len(own)), replace=False)
    en = mesh.ele_nodes
    flat = en.ravel()
    order = np.argsort(flat, kind="stable")
    starts = np.searchsorted(flat[order], sample)
    ends = np.searchsorted(flat[order], sample, side="right")
    fscale = np.abs(fint_lib).max()
    worst = 0.0
    for nd, s0, s1 in zip(sample, starts, ends):
        fi = np.zeros(3)
        for k in order[s0:s1]:
            e, a_loc = divmod(int(k), 27)
            nodes = en[e]
            Xe = X[nodes]
            ue = np.stack([uh[mesh.node_dof_row[m] + np.arange(3)] if mesh.node_dof_row[m] >= 0 else
                           np.zeros(3) for m in nodes])
            err, _, fe = orc.solid_evaluate(orc.HEX27, orc.TOTLAG, E, NU, Xe, ue, want_k=False)
            assert err == 0
            fi += fe[3 * a_loc:3 * a_loc + 3]
        r = fi - fext[mesh.node_dof_row[nd] + np.arange(3)]
        worst = max(worst, np.abs(r).max() / fscale)
    assert worst <= 1e-9, worst
