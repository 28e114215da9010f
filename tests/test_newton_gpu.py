"""The Newton path on the device: Dirichlet rows, CSR operator, block-Jacobi PCG
and the static Newton driver (4c_amd/newton.py), against
  * the reference's own RESULT DESCRIPTION values (the three known-answer inputs the oracle is
    pinned on) -- assembled, constrained and solved entirely through the library;
  * scipy on the oracle's assembly for box meshes (config 1's cantilever Newton step, a
    TotLag multi-iteration case on the structured sweep path).
Tolerances: RESULT values at the reference's own tolerances; solutions vs the direct solve at
1e-8 relative (the PCG stops at |r| <= 1e-13 |b|)."""

import importlib
import json
import os

import numpy as np
import pytest

import fixture_problem as fp
from parity_util import oracle_evaluate, rel_err

fcg = importlib.import_module("4c_amd").fcg
newton = importlib.import_module("4c_amd.newton")
torch = pytest.importorskip("torch")
sp = pytest.importorskip("scipy.sparse")
spla = pytest.importorskip("scipy.sparse.linalg")

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
E, NU = 210.0, 0.3


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


@pytest.mark.parametrize("name", ["solid_ele_hex8_Standard_linear.json",
                                  "solid_ele_hex27_Standard_linear.json",
                                  "sohex27_patchtest_nl_cost_drt.json"])
def test_result_description_on_device(name):
    _dev()
    fx = json.load(open(os.path.join(GOLD, name)))
    prob = fp.problem(fx)
    dis = fp.discretization(prob)
    ev = fcg.Evaluator(dis, kinematics=fp.kinematics_of(fx), youngs=prob.E, poisson=prob.nu)
    t = fp.end_time(fx)
    nt = newton.StaticNewton(ev, fp.fext(prob, t), prob.dirichlet_dofs(), tol_res=1e-11,
                             tol_inc=1e-12)
    u = nt.solve().cpu().numpy()
    for r in fx["results"]:
        got = u[3 * prob.lid[r["node"]] + r["dof"]]
        assert abs(got - r["value"]) <= r["tol"], (r, got, nt.history)


def test_result_description_structured_sweep():
    """The reference's hex8 known answer through the structured row-block sweep (lattice hint)."""
    _dev()
    fx = json.load(open(os.path.join(GOLD, "solid_ele_hex8_Standard_linear.json")))
    prob = fp.problem(fx)
    dis = fp.discretization(prob, lattice=True)
    ev = fcg.Evaluator(dis, kinematics=fcg.LINEAR, youngs=prob.E, poisson=prob.nu,
                       path=fcg.PATH_STRUCTURED)
    assert ev.info.path == fcg.PATH_STRUCTURED
    nt = newton.StaticNewton(ev, fp.fext(prob, fp.end_time(fx)), prob.dirichlet_dofs(),
                             tol_res=1e-11, tol_inc=1e-12)
    u = nt.solve().cpu().numpy()
    for r in fx["results"]:
        got = u[3 * prob.lid[r["node"]] + r["dof"]]
        assert abs(got - r["value"]) <= r["tol"], (r, got, nt.history)


def _cantilever(iv=(10, 10, 10), upper=(10.0, 1.0, 1.0)):
    mesh = fcg.BoxMesh(fcg.HEX8, iv, upper=upper)
    # x- face: all DOFs fixed; x+ face: surface load (0, 0, -1e-3)
    X = mesh.node_x
    dbc_nodes = np.nonzero(np.isclose(X[:, 0], 0.0) & (mesh.node_dof_row >= 0))[0]
    dbc = np.sort((mesh.node_dof_row[dbc_nodes][:, None] + np.arange(3)).ravel()).astype(np.int32)
    faces = []
    for e, (i, j, k) in enumerate(mesh.ele_ijk):
        if i == iv[0] - 1:
            faces.append(mesh.ele_nodes[e][[1, 2, 6, 5]])
    fext = np.zeros(mesh.n_rows)
    fcg.neumann_surface(fcg.HEX8, np.array(faces), X, mesh.node_dof_row, [1, 1, 1],
                        [0.0, 0.0, -1e-3], fext)
    return mesh, dbc, fext


def _cpu_newton(mesh, kinem, dbc, fext, iters):
    u = np.zeros(mesh.n_cols)
    free = np.setdiff1d(np.arange(mesh.n_rows), dbc)
    for _ in range(iters):
        err, _, K, f = oracle_evaluate(mesh, kinem, E, NU, u)
        assert err == 0
        A = sp.csr_matrix((K, mesh.col_lid, mesh.rowptr), shape=(mesh.n_rows, mesh.n_cols))
        r = f - fext
        du = spla.spsolve(A[free][:, free].tocsc(), -r[free])
        u[free] += du
    return u


def test_cantilever_newton_step_config1():
    _dev()
    mesh, dbc, fext = _cantilever()
    ev = fcg.Evaluator(mesh, kinematics=fcg.LINEAR, youngs=E, poisson=NU)
    assert ev.info.path == fcg.PATH_STRUCTURED
    nt = newton.StaticNewton(ev, fext, dbc, tol_res=1e-9, tol_inc=1e-9, lin_rtol=1e-14)
    u = nt.solve().cpu().numpy()
    ref = _cpu_newton(mesh, fcg.LINEAR, dbc, fext, 1)
    assert rel_err(u, ref) <= 1e-8, rel_err(u, ref)
    # linear: one step; the PCG tolerance may leave a rounding-level correction step
    assert len(nt.history) <= 3, nt.history
    assert all(h["norm_inc"] <= 1e-9 * nt.history[1]["norm_inc"] for h in nt.history[2:])
    assert np.all(u[dbc] == 0.0)


def test_totlag_newton_structured():
    _dev()
    mesh, dbc, fext = _cantilever(iv=(6, 3, 3), upper=(6.0, 1.0, 1.0))
    fext *= 2e3  # large tip load -> several Newton iterations
    ev = fcg.Evaluator(mesh, kinematics=fcg.TOTLAG, youngs=E, poisson=NU)
    nt = newton.StaticNewton(ev, fext, dbc, tol_res=1e-10, tol_inc=1e-10, lin_rtol=1e-14)
    u = nt.solve().cpu().numpy()
    n_it = len(nt.history) - 1
    assert n_it >= 3, nt.history
    ref = _cpu_newton(mesh, fcg.TOTLAG, dbc, fext, n_it)
    assert rel_err(u, ref) <= 1e-8, (rel_err(u, ref), nt.history)


def test_rescue_bad_newton_solve_continues_with_truncated_solves():
    """NOX "Rescue Bad Newton Solve" (4C default true, 4C_inpar_solver_nonlin.cpp:65-69): PCG
    capped at 60 % of the iterations the exact solves take never reaches its tolerance, Newton
    keeps the inexact directions (each step marked) and still converges to the exact-solve
    displacement; with the rescue off the first truncated solve raises."""
    _dev()
    mesh, dbc, fext = _cantilever(iv=(6, 3, 3), upper=(6.0, 1.0, 1.0))
    fext *= 2e3
    ev = fcg.Evaluator(mesh, kinematics=fcg.TOTLAG, youngs=E, poisson=NU)
    exact = newton.StaticNewton(ev, fext, dbc, tol_res=1e-10, tol_inc=1e-10, lin_rtol=1e-14)
    u_ref = exact.solve().cpu().numpy()
    cap = max(10, int(0.6 * max(h["lin_iter"] for h in exact.history if "lin_iter" in h)))
    nt = newton.StaticNewton(ev, fext, dbc, tol_res=1e-8, tol_inc=1e-8, max_iter=200,
                             lin_rtol=1e-14, lin_max_iter=cap)
    with pytest.warns(RuntimeWarning, match="Rescue Bad Newton Solve"):
        u = nt.solve().cpu().numpy()
    assert sum(1 for h in nt.history if h.get("lin_rescued")) >= 2, nt.history
    assert all(h["lin_iter"] <= cap for h in nt.history if "lin_iter" in h)
    assert rel_err(u, u_ref) <= 1e-6, rel_err(u, u_ref)
    strict = newton.StaticNewton(ev, fext, dbc, lin_rtol=1e-14, lin_max_iter=cap,
                                 rescue_bad_newton_solve=False)
    with pytest.raises(RuntimeError, match="above its tolerance"):
        strict.solve()


@pytest.mark.parametrize("method", ["Type 1", "Type 2"])
def test_inexact_newton_forcing_term_same_solution(method):
    """NOX forcing terms (newton.ForcingTerm): looser early linear solves, same converged u."""
    _dev()
    mesh, dbc, fext = _cantilever(iv=(6, 3, 3), upper=(6.0, 1.0, 1.0))
    fext *= 2e3
    ev = fcg.Evaluator(mesh, kinematics=fcg.TOTLAG, youngs=E, poisson=NU)
    exact = newton.StaticNewton(ev, fext, dbc, tol_res=1e-10, tol_inc=1e-10, lin_rtol=1e-14)
    u_ref = exact.solve().cpu().numpy()
    nt = newton.StaticNewton(ev, fext, dbc, tol_res=1e-10, tol_inc=1e-10, max_iter=40,
                             forcing=newton.ForcingTerm(method))
    u = nt.solve().cpu().numpy()
    assert rel_err(u, u_ref) <= 1e-9, (rel_err(u, u_ref), nt.history)
    etas = [h["eta"] for h in nt.history if "eta" in h]
    assert etas[0] == 0.1 and all(1e-6 <= e <= 0.01 for e in etas[1:]), etas
    lin = sum(h["lin_iter"] for h in nt.history if "lin_iter" in h)
    lin_exact = sum(h["lin_iter"] for h in exact.history if "lin_iter" in h)
    assert lin < lin_exact, (lin, lin_exact)


def test_spmv_dirichlet_pcg_against_scipy():
    dev = _dev()
    mesh = fcg.BoxMesh(fcg.HEX8, (8, 6, 5), jitter=0.1)
    ev = fcg.Evaluator(mesh, kinematics=fcg.LINEAR, youngs=E, poisson=NU)
    u = torch.from_numpy(mesh.u_col(1e-3)).to(dev)
    f = torch.zeros(mesh.n_rows, dtype=torch.float64, device=dev)
    K = torch.zeros(mesh.nnz, dtype=torch.float64, device=dev)
    ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, u, f, K)
    Kh = K.cpu().numpy()
    A = sp.csr_matrix((Kh, mesh.col_lid, mesh.rowptr), shape=(mesh.n_rows, mesh.n_cols))
    x = np.random.default_rng(3).standard_normal(mesh.n_cols)
    y = torch.empty(mesh.n_rows, dtype=torch.float64, device=dev)
    ev.spmv(K, torch.from_numpy(x).to(dev), y)
    assert rel_err(y.cpu().numpy(), A @ x) <= 1e-14
    # Dirichlet rows on the bottom face, reactions extracted, then PCG vs direct solve
    dbc = np.nonzero(np.isclose(np.repeat(mesh.node_x[:, 2], 3), 0.0))[0].astype(np.int32)
    rhs = torch.from_numpy(np.random.default_rng(4).standard_normal(mesh.n_rows)).to(dev)
    rhs_h = rhs.cpu().numpy().copy()
    freact = torch.zeros_like(rhs)
    ev.dirichlet_apply(torch.from_numpy(dbc).to(dev), K, rhs, freact)
    Kd = K.cpu().numpy()
    rows = np.repeat(np.arange(mesh.n_rows), np.diff(mesh.rowptr))
    isd = np.isin(rows, dbc)
    assert np.all(Kd[isd & (mesh.col_lid == rows)] == 1.0)
    assert np.all(Kd[isd & (mesh.col_lid != rows)] == 0.0)
    assert np.array_equal(Kd[~isd], Kh[~isd])
    assert np.array_equal(freact.cpu().numpy()[dbc], -rhs_h[dbc])  # extract_freact scales by -1
    assert np.all(rhs.cpu().numpy()[dbc] == 0.0)
    sol = torch.empty_like(rhs)
    it, rr = ev.pcg_solve(K, rhs, sol, rtol=1e-14, max_iter=5000)
    assert rr <= 1e-13, (it, rr)
    Ad = sp.csr_matrix((Kd, mesh.col_lid, mesh.rowptr), shape=(mesh.n_rows, mesh.n_cols))
    ref = spla.spsolve(Ad.tocsc(), rhs.cpu().numpy())
    assert rel_err(sol.cpu().numpy(), ref) <= 1e-9
    # bitwise reproducible
    sol2 = torch.empty_like(rhs)
    ev.pcg_solve(K, rhs, sol2, rtol=1e-14, max_iter=5000)
    assert torch.equal(sol, sol2)


@pytest.mark.parametrize("name", ["solid_ele_hex8_Standard_eas_none_volume_neumann.json",
                                  "solid_ele_hex27_Standard_volume_neumann.json"])
def test_neohooke_result_description_on_device(name):
    """ElastHyper/CoupNeoHooke, large deformation (|u| ~ 2.9), the reference's two load steps;
    every tangent and residual from the library, Newton solved on the host."""
    dev = _dev()
    fx = json.load(open(os.path.join(GOLD, name)))
    prob = fp.problem(fx)
    dis = fp.discretization(prob)
    ev = fcg.Evaluator(dis, kinematics=fcg.TOTLAG, youngs=prob.E, poisson=prob.nu,
                       material=fcg.MAT_ELASTHYPER_COUPNEOHOOKE)

    def assemble(u):
        f = torch.zeros(dis.n_rows, dtype=torch.float64, device=dev)
        K = torch.zeros(dis.nnz, dtype=torch.float64, device=dev)
        ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, torch.from_numpy(u).to(dev), f, K)
        D = np.zeros((dis.n_rows, dis.n_cols))
        rows = np.repeat(np.arange(dis.n_rows), np.diff(dis.rowptr))
        D[rows, dis.col_lid] = K.cpu().numpy()
        return D, f.cpu().numpy()

    t = fp.end_time(fx)
    dt = float(fx["dynamic"]["TIMESTEP"])
    u = prob.solve_statics(t=t, nsteps=int(round(t / dt)), assemble=assemble)
    for r in fx["results"]:
        got = prob.disp(u, r["node"], r["dof"])
        assert abs(got - r["value"]) <= r["tol"], (r, got)


# ------------------------------------------------- reactions, analytical error, DOMAIN (device)
import known_answers as ka  # noqa: E402


@pytest.mark.parametrize("name", ["patch_test_cube_linear_test_react.json",
                                  "patch_test_cube_h27_linear_test_react.json"])
def test_reaction_forces_on_device(name):
    """Reaction forces of patch_test_cube_*_linear_test_react.dat (1e-13) from the library alone:
    StaticNewton's final evaluate + fcg_dirichlet_apply (extract_freact's -F at the DBC rows)."""
    _dev()
    fx = json.load(open(os.path.join(GOLD, name)))
    prob = fp.problem(fx)
    dis = fp.discretization(prob)
    ev = fcg.Evaluator(dis, kinematics=fp.kinematics_of(fx), youngs=prob.E, poisson=prob.nu)
    nt = newton.StaticNewton(ev, fp.fext(prob, 1.0), prob.dirichlet_dofs(), tol_res=1e-12,
                             tol_inc=1e-13, lin_rtol=1e-14)
    u = nt.solve().cpu().numpy()
    for r in fx["results"]:
        assert abs(u[3 * prob.lid[r["node"]] + r["dof"]] - r["value"]) <= r["tol"], r
    assert ka.check_reactions(fx, prob, nt.freact.cpu().numpy()) == []


@pytest.mark.parametrize("lattice", [False, True])
def test_analytical_error_cantilever_on_device(lattice):
    """error_analytical_beam_cantilever_end_surface_load_with_poissons_effect.dat through the
    library (general path, and the structured sweep via the lattice hint the beam admits): the
    RESULT DESCRIPTION (1e-10) and the L2-error CSV (rtol 1e-10, atol 1e-12)."""
    _dev()
    fx = json.load(open(os.path.join(GOLD,
                    "error_analytical_beam_cantilever_end_surface_load_with_poissons_effect.json")))
    prob = fp.problem(fx)
    dis = fp.discretization(prob, lattice=lattice)
    ev = fcg.Evaluator(dis, kinematics=fcg.LINEAR, youngs=prob.E, poisson=prob.nu,
                       path=fcg.PATH_STRUCTURED if lattice else fcg.PATH_GENERAL)
    assert ev.info.path == (fcg.PATH_STRUCTURED if lattice else fcg.PATH_GENERAL)
    nt = newton.StaticNewton(ev, fp.fext(prob, 1.0), prob.dirichlet_dofs(), tol_res=1e-12,
                             tol_inc=1e-12, lin_rtol=1e-14)
    u = nt.solve().cpu().numpy()
    for r in fx["results"]:
        assert abs(u[3 * prob.lid[r["node"]] + r["dof"]] - r["value"]) <= r["tol"], r
    ref = dict(zip(fx["csv_reference"]["columns"], fx["csv_reference"]["rows"][0]))
    tol = fx["csv_tolerance"]
    for k, v in zip(("displacement_error_l2_norm", "displacement_integral", "reference_volume"),
                    ka.analytical_error(fx, prob, u)):
        assert abs(v - ref[k]) <= tol["atol"] + tol["rtol"] * abs(ref[k]), (k, v, ref[k])


@pytest.mark.parametrize("nranks", [1, 2])
def test_domain_altgeogeneration_on_device(nranks):
    """sohex8_disp_altgeogeneration.dat (STRUCTURE DOMAIN, NP 2 in the reference): the box of
    fcg_box_mesh_create at 1 and 2 ranks, every rank's owned K rows from its own context on the
    device (structured sweep), gathered by DOF GID; NODE 49 (GID 48) dispx = 4.0 at 1e-14."""
    dev = _dev()
    fx = json.load(open(os.path.join(GOLD, "sohex8_disp_altgeogeneration.json")))
    meshes = ka.domain_meshes(fx, nranks)
    E, nu = fx["material"]["young"], fx["material"]["nue"]

    def assemble(m, u):
        ev = fcg.Evaluator(m, kinematics=fcg.TOTLAG, youngs=E, poisson=nu)
        assert ev.info.path == fcg.PATH_STRUCTURED
        f = torch.zeros(m.n_rows, dtype=torch.float64, device=dev)
        K = torch.full((m.nnz,), float("nan"), dtype=torch.float64, device=dev)
        ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, torch.from_numpy(u).to(dev), f, K)
        return K.cpu().numpy(), f.cpu().numpy()

    u = ka.domain_solve(fx, meshes, assemble)
    assert ka.check_domain_results(fx, u) == []
