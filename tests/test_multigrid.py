"""Geometric multigrid preconditioner of the Newton solve (4c_amd/multigrid.py).

Host (no GPU): the transfer tables of GridGenerator boxes -- hex27 -> hex8 on the same elements,
hex8 n -> n/2 and the non-nested odd n -> (n + 1)/2 -- interpolate linear fields exactly and the restriction is the transpose of the
prolongation.  GPU: fcg_node_transfer and fcg_block_jacobi_apply against numpy on the same tables,
and Newton solves with the multigrid-preconditioned flexible CG converging to the block-Jacobi
PCG's displacement (the preconditioner changes the path, not the solution: 1e-8 relative at
linear tolerance 1e-12) in far fewer iterations."""

import importlib

import numpy as np
import pytest

fcg = importlib.import_module("4c_amd").fcg
mgm = importlib.import_module("4c_amd.multigrid")
newton = importlib.import_module("4c_amd.newton")

E, NU = 210.0, 0.3


def _apply(tab, x, n):
    ptr, src, w, dst = tab
    y = np.zeros(n)
    for o in range(len(dst)):
        if dst[o] < 0:
            continue
        acc = np.zeros(3)
        for j in range(ptr[o], ptr[o + 1]):
            acc += w[j] * x[src[j]:src[j] + 3]
        y[dst[o]:dst[o] + 3] = acc
    return y


def _pairs():
    up = (2.0, 1.0, 3.0)
    f27 = fcg.BoxMesh(fcg.HEX27, (4, 2, 6), upper=up)
    c8 = fcg.BoxMesh(fcg.HEX8, (4, 2, 6), upper=up)
    c8h = fcg.BoxMesh(fcg.HEX8, (2, 1, 3), upper=up)
    # odd interval counts halved to (n + 1) / 2: a non-nested coarse level
    o8 = fcg.BoxMesh(fcg.HEX8, (5, 3, 7), upper=up)
    o8h = fcg.BoxMesh(fcg.HEX8, (3, 2, 4), upper=up)
    return [(f27, c8), (c8, c8h), (o8, o8h)]


@pytest.mark.parametrize("k", [0, 1, 2])
def test_transfer_tables_host(k):
    fine, coarse = _pairs()[k]
    P, R = mgm.transfer_tables(fine, coarse)
    A = np.array([[1.0, 2.0, 3.0], [0.5, -1.0, 2.0], [3.0, 1.0, -2.0]])
    xc, xf = np.zeros(coarse.n_rows), np.zeros(fine.n_rows)
    for d in range(3):
        xc[coarse.node_dof_row + d] = coarse.node_x @ A[d] + d
        xf[fine.node_dof_row + d] = fine.node_x @ A[d] + d
    assert np.abs(_apply(P, xc, fine.n_rows) - xf).max() <= 1e-13
    rng = np.random.default_rng(7)
    a, b = rng.standard_normal(fine.n_rows), rng.standard_normal(coarse.n_rows)
    assert abs(a @ _apply(P, b, fine.n_rows) - b @ _apply(R, a, coarse.n_rows)) <= 1e-12 * (
        np.abs(a).sum() + np.abs(b).sum())
    # every fine node gets weights summing to one (partition of unity)
    ptr, _, w, _ = P
    assert np.allclose(np.add.reduceat(w, ptr[:-1]), 1.0)


def test_multigrid_rejects_meshes_without_a_hierarchy():
    m = fcg.BoxMesh(fcg.HEX8, (3, 3, 3))
    with pytest.raises(ValueError):
        mgm.Multigrid(m, None, lambda mm: np.zeros(mm.n_node, bool), E, NU)
    with pytest.raises(ValueError):
        mgm.Multigrid(object(), None, None, E, NU)


def test_matrix_free_fine_level_needs_hex27_fp64():
    """Multigrid(matrix_free=True) applies fcg_tangent_apply (hex27 only) and is exact FP64: a hex8
    fine level or mixed=True is refused before any device work."""
    m8 = fcg.BoxMesh(fcg.HEX8, (4, 4, 4))
    m27 = fcg.BoxMesh(fcg.HEX27, (4, 4, 4))
    with pytest.raises(ValueError):
        mgm.Multigrid(m8, None, lambda mm: np.zeros(mm.n_node, bool), E, NU, matrix_free=True)
    with pytest.raises(ValueError):
        mgm.Multigrid(m27, None, lambda mm: np.zeros(mm.n_node, bool), E, NU, matrix_free=True,
                      mixed=True)
    with pytest.raises(ValueError):  # the outer operator matrix-free needs the fine level's action
        mgm.Multigrid(m27, None, lambda mm: np.zeros(mm.n_node, bool), E, NU, outer_matrix_free=True)


def _dev():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch, torch.device("cuda:0")


@pytest.mark.gpu
@pytest.mark.parametrize("k", [0, 1, 2])
def test_node_transfer_device(k):
    torch, dev = _dev()
    fine, coarse = _pairs()[k]
    P, R = mgm.transfer_tables(fine, coarse)
    rng = np.random.default_rng(3)
    xc, xf = rng.standard_normal(coarse.n_rows), rng.standard_normal(fine.n_rows)
    for tab, x, n in ((P, xc, fine.n_rows), (R, xf, coarse.n_rows)):
        t = mgm._Transfer(tab, dev)
        y = torch.full((n,), 5.0, dtype=torch.float64, device=dev)
        t(torch.from_numpy(x).to(dev), y, accumulate=True)
        ref = _apply(tab, x, n) + 5.0
        torch.cuda.synchronize()
        assert np.abs(y.cpu().numpy() - ref).max() <= 1e-13 * max(1.0, np.abs(ref).max())


@pytest.mark.gpu
@pytest.mark.parametrize("k", [0, 1])
def test_box_transfer_matches_tables(k):
    """fcg_box_transfer (implicit 2:1 weights, the level masks in the kernel) = fcg_node_transfer on
    the tables followed by the mask, both directions, with clamped nodes on both levels."""
    torch, dev = _dev()
    fine, coarse = _pairs()[k]
    P, R = mgm.transfer_tables(fine, coarse)

    def dbc(m):
        nodes = np.nonzero(mgm.node_lattice(m)[:, 0] == 0)[0]
        return np.sort((m.node_dof_row[nodes][:, None] + np.arange(3)).ravel()).astype(np.int32)

    fr, cr = dbc(fine), dbc(coarse)
    bt = mgm._BoxTransfer(fine, fr, coarse, cr, dev)
    rng = np.random.default_rng(11)
    xc = torch.from_numpy(rng.standard_normal(coarse.n_rows)).to(dev)
    xf = torch.from_numpy(rng.standard_normal(fine.n_rows)).to(dev)
    mf = torch.ones(fine.n_rows, dtype=torch.float64, device=dev)
    mf[torch.as_tensor(fr.astype(np.int64), device=dev)] = 0.0
    mc = torch.ones(coarse.n_rows, dtype=torch.float64, device=dev)
    mc[torch.as_tensor(cr.astype(np.int64), device=dev)] = 0.0
    y0 = torch.full((fine.n_rows,), 3.0, dtype=torch.float64, device=dev)
    y1 = y0.clone()
    mgm._Transfer(P, dev)(xc, y0, accumulate=True)
    y0.mul_(mf)
    bt.prolong(xc, y1)
    b0 = torch.empty(coarse.n_rows, dtype=torch.float64, device=dev)
    b1 = torch.empty_like(b0)
    mgm._Transfer(R, dev)(xf, b0, accumulate=False)
    b0.mul_(mc)
    bt.restrict(xf, b1)
    torch.cuda.synchronize()
    for a, b in ((y0, y1), (b0, b1)):
        a, b = a.cpu().numpy(), b.cpu().numpy()
        assert np.abs(a - b).max() <= 1e-14 * max(1.0, np.abs(a).max())


def _cantilever(ct, n, kin, load, length=2.0, jitter=0.0):
    mesh = fcg.BoxMesh(ct, (n, n, n), upper=(length, 1.0, 1.0), jitter=jitter)
    X = mesh.node_x
    clamp = lambda m: np.isclose(m.node_x[:, 0], 0.0)  # noqa: E731
    nodes = np.nonzero(clamp(mesh))[0]
    dbc = np.sort((mesh.node_dof_row[nodes][:, None] + np.arange(3)).ravel()).astype(np.int32)
    face = [1, 2, 6, 5] if ct == fcg.HEX8 else [1, 2, 6, 5, 9, 14, 17, 13, 22]
    faces = mesh.ele_nodes[mesh.ele_ijk[:, 0] == n - 1][:, face]
    fext = np.zeros(mesh.n_rows)
    fcg.neumann_surface(ct, faces, X, mesh.node_dof_row, [1, 1, 1], [0.0, 0.0, load], fext)
    return mesh, clamp, dbc, fext


@pytest.mark.gpu
@pytest.mark.parametrize("iv,rot", [((5, 4, 3), (0.0, 0.0, 0.0)), ((3, 6, 2), (0.3, -0.2, 0.5))])
def test_box_stencil_matches_assembled_operator(iv, rot):
    """fcg_box_stencil_apply (the coarse levels' operator) = fcg_spmv on the same box's assembled,
    Dirichlet-modified K, every node class (faces, edges, corners, interior) and unit rows."""
    torch, dev = _dev()
    mesh = fcg.BoxMesh(fcg.HEX8, iv, upper=(2.0, 1.0, 1.5), rotation=rot)
    clamp = np.isclose(mgm.node_lattice(mesh)[:, 0], 0)
    nodes = np.nonzero(clamp)[0]
    rows = np.sort((mesh.node_dof_row[nodes][:, None] + np.arange(3)).ravel()).astype(np.int32)
    ev = fcg.Evaluator(mesh, kinematics=fcg.LINEAR, youngs=E, poisson=NU)
    f64 = dict(dtype=torch.float64, device=dev)
    K = torch.zeros(mesh.nnz, **f64)
    ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, torch.zeros(mesh.n_cols, **f64),
                       torch.zeros(mesh.n_rows, **f64), K)
    ev.dirichlet_apply(torch.as_tensor(rows, device=dev), K)
    lvl = mgm._Level(mesh, ev, K, rows, dev)
    x = torch.from_numpy(np.random.default_rng(2).standard_normal(mesh.n_rows)).to(dev)
    y0, y1 = torch.empty_like(x), torch.empty_like(x)
    lvl.spmv_exact(x, y0)
    lvl.stencil = mgm.box_stencil(mesh, E, NU, dev, rows)
    assert lvl.stencil is not None
    lvl.spmv_exact(x, y1)
    torch.cuda.synchronize()
    a, b = y0.cpu().numpy(), y1.cpu().numpy()
    assert np.linalg.norm(a - b) <= 1e-13 * np.linalg.norm(a)
    assert np.array_equal(b[rows], x.cpu().numpy()[rows])
    ev.close()


@pytest.mark.gpu
def test_block_jacobi_apply_device():
    torch, dev = _dev()
    mesh, clamp, dbc, fext = _cantilever(fcg.HEX8, 4, fcg.LINEAR, -1e-2)
    ev = fcg.Evaluator(mesh, kinematics=fcg.LINEAR, youngs=E, poisson=NU)
    f64 = dict(dtype=torch.float64, device=dev)
    K = torch.zeros(mesh.nnz, **f64)
    ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, torch.zeros(mesh.n_cols, **f64),
                       torch.zeros(mesh.n_rows, **f64), K)
    lvl = mgm._Level(mesh, ev, K, dbc, dev)
    lvl.setup_diag()
    r = np.random.default_rng(5).standard_normal(mesh.n_rows)
    z = torch.ones(mesh.n_rows, **f64)
    lvl.apply_dinv(torch.from_numpy(r).to(dev), z, 0.5, accumulate=True)
    torch.cuda.synchronize()
    Kh, rp, ci = K.cpu().numpy(), mesh.rowptr, mesh.col_lid
    ref = np.ones(mesh.n_rows)
    for node in range(mesh.n_node):
        i = mesh.node_dof_row[node]
        D = np.zeros((3, 3))
        for a in range(3):
            for j in range(rp[i + a], rp[i + a + 1]):
                if i <= ci[j] < i + 3:
                    D[a, ci[j] - i] = Kh[j]
        ref[i:i + 3] += 0.5 * np.linalg.solve(D, r[i:i + 3])
    assert np.abs(z.cpu().numpy() - ref).max() <= 1e-12 * np.abs(ref).max()


@pytest.mark.gpu
@pytest.mark.parametrize("ct,n,kin,load,length,jitter,tol", [
    (fcg.HEX27, 6, fcg.TOTLAG, -2.0, 2.0, 0.0, 1e-10),
    (fcg.HEX8, 8, fcg.LINEAR, -1e-2, 2.0, 0.0, 1e-10),
    (fcg.HEX8, 8, fcg.TOTLAG, -2.0, 2.0, 0.0, 1e-10),
    # BASELINE config 1's cantilever (10 x 10 x 10 hex8 over [0,10] x [0,1]^2, aspect ratio 10:
    # its round-off floor sits near 1e-10 |f_ext|, so the Newton tolerance is looser)
    (fcg.HEX8, 10, fcg.LINEAR, -1.0, 10.0, 0.0, 1e-8),
    # jittered interior nodes: the coarse levels stay unjittered (a preconditioner only)
    (fcg.HEX8, 8, fcg.LINEAR, -1.0, 1.0, 0.1, 1e-10)])
def test_newton_multigrid_matches_pcg(ct, n, kin, load, length, jitter, tol):
    torch, dev = _dev()
    mesh, clamp, dbc, fext = _cantilever(ct, n, kin, load, length, jitter)
    tol_res = tol * np.linalg.norm(fext)
    res = {}
    for name in ("pcg", "mg"):
        ev = fcg.Evaluator(mesh, kinematics=kin, youngs=E, poisson=NU)
        mg = mgm.Multigrid(mesh, ev, clamp, E, NU, min_intervals=2) if name == "mg" else None
        nt = newton.StaticNewton(ev, fext, dbc, tol_res=tol_res, tol_inc=1e-9, lin_rtol=1e-12,
                                 linear_solver=mg)
        u = nt.solve()
        res[name] = (u.cpu().numpy(), sum(h.get("lin_iter", 0) for h in nt.history),
                     len(nt.history), mg.describe() if mg else None)
        ev.close()
    (u0, it0, n0, _), (u1, it1, n1, lv) = res["pcg"], res["mg"]
    assert len(lv) >= 2
    assert np.linalg.norm(u1 - u0) <= 100 * tol * np.linalg.norm(u0)
    # per linear solve: on the aspect-ratio-10 case the Newton's last steps solve round-off
    # residuals, and how many of them it takes to meet tol_inc is not the preconditioner's doing
    assert it1 / (n1 - 1) * 3 < it0 / (n0 - 1), (it0, n0, it1, n1)


@pytest.mark.gpu
def test_multigrid_pre_smoothing_only_on_the_finest_level():
    """fine_post=False: a nonsymmetric V-cycle (no fine post-smoothing), which the flexible CG
    admits -- same Newton solution, every linear solve converged."""
    torch, dev = _dev()
    mesh, clamp, dbc, fext = _cantilever(fcg.HEX8, 8, fcg.TOTLAG, -2.0)
    res = {}
    for post in (True, False):
        ev = fcg.Evaluator(mesh, kinematics=fcg.TOTLAG, youngs=E, poisson=NU)
        mg = mgm.Multigrid(mesh, ev, clamp, E, NU, min_intervals=2, fine_post=post)
        nt = newton.StaticNewton(ev, fext, dbc, tol_res=1e-10 * np.linalg.norm(fext), tol_inc=1e-9,
                                 lin_rtol=1e-10, linear_solver=mg)
        res[post] = nt.solve().cpu().numpy()
        ev.close()
    assert np.linalg.norm(res[False] - res[True]) <= 1e-8 * np.linalg.norm(res[True])


@pytest.mark.gpu
@pytest.mark.parametrize("ct", [fcg.HEX8, fcg.HEX27])
def test_fused_chebyshev_step_is_bit_identical(monkeypatch, ct):
    """fcg_chebyshev_step (r = b - y, d = c_d d + c_r D^-1 r, x += d in one pass) against the
    separate torch / block-Jacobi passes: the same Newton iterates bit for bit."""
    torch, dev = _dev()
    mesh, clamp, dbc, fext = _cantilever(ct, 6, fcg.TOTLAG, -2.0)
    res = {}
    for fused in ("1", "0"):
        monkeypatch.setenv("FCG_MG_FUSED", fused)
        ev = fcg.Evaluator(mesh, kinematics=fcg.TOTLAG, youngs=E, poisson=NU)
        mg = mgm.Multigrid(mesh, ev, clamp, E, NU, min_intervals=2)
        nt = newton.StaticNewton(ev, fext, dbc, tol_res=1e-10 * np.linalg.norm(fext), tol_inc=1e-9,
                                 lin_rtol=1e-10, linear_solver=mg)
        res[fused] = (nt.solve().cpu().numpy(), [h.get("lin_iter") for h in nt.history])
        ev.close()
    assert res["1"][1] == res["0"][1]
    assert np.array_equal(res["1"][0], res["0"][0])


@pytest.mark.gpu
def test_multigrid_with_native_amg_coarsest_level():
    """coarse_solver="amg": the coarsest hex8 level solved by the native AMG set up once."""
    torch, dev = _dev()
    mesh, clamp, dbc, fext = _cantilever(fcg.HEX27, 8, fcg.TOTLAG, -2.0)
    res = {}
    for cs in ("pcg", "amg"):
        ev = fcg.Evaluator(mesh, kinematics=fcg.TOTLAG, youngs=E, poisson=NU)
        mg = mgm.Multigrid(mesh, ev, clamp, E, NU, min_intervals=2, coarse_solver=cs)
        nt = newton.StaticNewton(ev, fext, dbc, tol_res=1e-10 * np.linalg.norm(fext), tol_inc=1e-9,
                                 lin_rtol=1e-10, linear_solver=mg)
        res[cs] = (nt.solve().cpu().numpy(), [h.get("lin_iter") for h in nt.history])
        if mg.coarse_amg is not None:
            mg.coarse_amg.close()
        ev.close()
    (u0, it0), (u1, it1) = res["pcg"], res["amg"]
    assert np.linalg.norm(u1 - u0) <= 1e-8 * np.linalg.norm(u0)
    assert sum(i or 0 for i in it1) <= 1.5 * sum(i or 0 for i in it0), (it0, it1)
    with pytest.raises(ValueError):
        mgm.Multigrid(mesh, None, clamp, E, NU, coarse_solver="lu")


@pytest.mark.gpu
def test_stale_lmax_restarts_and_dirichlet_mismatch_raises():
    """a too-low kept lambda_max estimate is re-estimated and the solve restarted (the
    restart path), and a multigrid mask that disagrees with the Newton's Dirichlet rows is refused."""
    torch, dev = _dev()
    mesh, clamp, dbc, fext = _cantilever(fcg.HEX8, 8, fcg.LINEAR, -1e-2)
    ev = fcg.Evaluator(mesh, kinematics=fcg.LINEAR, youngs=E, poisson=NU)
    mg = mgm.Multigrid(mesh, ev, clamp, E, NU, min_intervals=2)
    with pytest.raises(ValueError):
        newton.StaticNewton(ev, fext, dbc[3:], linear_solver=mg)
    nt = newton.StaticNewton(ev, fext, dbc, tol_res=1e-10 * np.linalg.norm(fext), tol_inc=1e-9,
                             lin_rtol=1e-12, linear_solver=mg)
    u_ref = nt.solve().cpu().numpy()
    good = mg.levels[0].lmax
    mg.levels[0].lmax = 1e-3 * good  # stale and far too low
    u = nt.solve().cpu().numpy()
    assert mg.levels[0].lmax > 0.5 * good  # re-estimated
    assert np.linalg.norm(u - u_ref) <= 1e-8 * np.linalg.norm(u_ref)


@pytest.mark.gpu
def test_pcg_reports_breakdown_and_nonfinite():
    """fcg_pcg_solve returns FCG_ERR_SINGULAR for a non-finite system or a
    p.Kp <= 0 breakdown instead of FCG_OK with NaN."""
    torch, dev = _dev()
    mesh, clamp, dbc, fext = _cantilever(fcg.HEX8, 4, fcg.LINEAR, -1e-2)
    ev = fcg.Evaluator(mesh, kinematics=fcg.LINEAR, youngs=E, poisson=NU)
    f64 = dict(dtype=torch.float64, device=dev)
    K = torch.zeros(mesh.nnz, **f64)
    ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, torch.zeros(mesh.n_cols, **f64),
                       torch.zeros(mesh.n_rows, **f64), K)
    ev.dirichlet_apply(torch.from_numpy(dbc).to(dev), K)
    b = torch.from_numpy(fext).to(dev)
    x = torch.empty_like(b)
    bn = b.clone()
    bn[5] = float("nan")
    with pytest.raises(fcg.FcgError) as ei:
        ev.pcg_solve(K, bn, x)
    assert ei.value.code == 2
    with pytest.raises(fcg.FcgError) as ei:
        ev.pcg_solve(-K, b, x)  # negative definite: p.Kp < 0 on the first step
    assert ei.value.code == 2
    it, rr = ev.pcg_solve(K, b, x, rtol=1e-12)
    assert rr <= 1e-12
