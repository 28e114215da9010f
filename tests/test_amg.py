"""Smoothed-aggregation AMG (4c_amd/amg.py, fcg_amg.hip, fcg_amg_setup.cpp; SURVEY §8f row 2 on
meshes without a box hierarchy).

Host (no GPU): aggregation covers every free node exactly once and skips the Dirichlet nodes; the
tentative factor is Q R = near-null space with orthonormal Q (rank-deficient aggregates give zero
columns); the symbolic product and transpose patterns equal scipy's.  GPU: every BSR kernel against
numpy on random blocks; the hierarchy against its definition (P = T - omega D^-1 A T and
A_c = P^T A P from dense numpy products); Newton solves on unstructured meshes (a renumbered box,
the reference's beam mesh tiled and jittered, hex27, TotLag) converge to the block-Jacobi PCG's
displacement in a fraction of the iterations.  The AMG changes the iteration path only: parity is
the PCG solution, MueLu itself being absent (parity of the preconditioner unpinned)."""

import importlib

import numpy as np
import pytest
import scipy.sparse as sp

from test_oracle_known_answers import load_fixture
from parity_util import tiled_input_mesh

fcg = importlib.import_module("4c_amd").fcg
amg = importlib.import_module("4c_amd.amg")
newton = importlib.import_module("4c_amd.newton")

E, NU = 210.0, 0.3
FX = "error_analytical_beam_cantilever_end_surface_load_with_poissons_effect.json"


def _block_graph(dis):
    nn = dis.n_rows // 3
    rp, cl = dis.rowptr, dis.col_lid
    r0 = rp[0:3 * nn:3]
    nb = (rp[1:3 * nn + 1:3] - r0) // 3
    bptr = np.concatenate([[0], np.cumsum(nb)]).astype(np.int64)
    off = np.arange(bptr[-1]) - np.repeat(bptr[:-1], nb)
    return bptr, (cl[np.repeat(r0, nb) + 3 * off] // 3).astype(np.int32)


def test_aggregation_covers_free_nodes_once():
    dis = fcg.Discretization.renumbered(fcg.BoxMesh(fcg.HEX8, (7, 5, 4)), seed=2)
    ptr, col = _block_graph(dis)
    n = len(ptr) - 1
    skip = np.isclose(dis.node_x[np.argsort(dis.node_dof_row)][:, 0], 0.0)
    agg, na = amg.aggregate(ptr, col, skip)
    assert (agg[skip] == -1).all() and (agg[~skip] >= 0).all()
    assert set(np.unique(agg[~skip])) == set(range(na))
    assert 0 < na < n // 4
    A = sp.csr_matrix((np.ones(len(col)), col, ptr), shape=(n, n))
    for a in range(na):  # every aggregate is connected in the graph
        idx = np.nonzero(agg == a)[0]
        sub = A[idx][:, idx]
        ncomp, _ = sp.csgraph.connected_components(sub, directed=False)
        assert ncomp == 1


def test_tentative_is_orthonormal_factor_of_the_modes():
    rng = np.random.default_rng(4)
    x = rng.standard_normal((40, 3))
    ns = amg.rigid_body_modes(x)
    agg = np.repeat(np.arange(8), 5).astype(np.int32)
    agg[39] = 7
    agg[35:39] = 7
    agg[30:35] = 6
    agg[0] = 8  # a singleton aggregate: 3 rows carry only 3 of the 6 modes
    agg = agg.astype(np.int32)
    na = 9
    tv, nsc, nd = amg.tentative(ns, agg, na)
    assert nd == 3
    for a in range(na):
        idx = np.nonzero(agg == a)[0]
        Q, M = tv[idx].reshape(-1, 6), ns[idx].reshape(-1, 6)
        assert np.abs(Q @ nsc[a] - M).max() <= 1e-13
        G = Q.T @ Q
        live = np.diag(G) > 0.5
        assert np.abs(G - np.diag(live.astype(float))).max() <= 1e-13
    # the coarse near-null space of a 6-DOF level factors the same way
    agg2 = np.array([0, 0, 1, 1, 1, 0, 1, 0, 1], dtype=np.int32)
    tv2, nsc2, _ = amg.tentative(nsc, agg2, 2)
    for a in range(2):
        idx = np.nonzero(agg2 == a)[0]
        assert np.abs(tv2[idx].reshape(-1, 6) @ nsc2[a] - nsc[idx].reshape(-1, 6)).max() <= 1e-12


def test_symbolic_and_transpose_patterns_match_scipy():
    rng = np.random.default_rng(9)
    A = sp.random(60, 45, density=0.08, random_state=1, format="csr")
    B = sp.random(45, 30, density=0.1, random_state=2, format="csr")
    p, c = amg.symbolic(A.indptr, A.indices, B.indptr, B.indices, 30)
    C = (abs(A) @ abs(B)).tocsr()
    C.eliminate_zeros()
    C.sort_indices()
    assert np.array_equal(p, C.indptr) and np.array_equal(c, C.indices)
    tp, tc, perm = amg.transpose_pattern(p, c, 30)
    T = C.T.tocsr()
    T.sort_indices()
    assert np.array_equal(tp, T.indptr) and np.array_equal(tc, T.indices)
    rows = np.repeat(np.arange(60), np.diff(p))
    assert np.array_equal(rows[perm], tc) and np.array_equal(c[perm], np.repeat(np.arange(30), np.diff(tp)))
    del rng


def test_product_plan_lists_the_pairs_in_row_order():
    """fcg_bsr_product_plan against a direct listing: per C block, the (A block, B block) pairs whose
    product lands on its column, in A's row order; a C pattern with a column dropped and one added
    (no product) lists none for them."""
    A = sp.random(40, 30, density=0.12, random_state=3, format="csr")
    B = sp.random(30, 25, density=0.15, random_state=4, format="csr")
    A.sort_indices()
    B.sort_indices()
    p, c = amg.symbolic(A.indptr, A.indices, B.indptr, B.indices, 25)
    rows = [list(c[p[i]:p[i + 1]]) for i in range(40)]
    rows[3] = rows[3][1:]  # drop a column
    rows[5] = sorted(set(rows[5]) | {24, 0})  # columns no product reaches (maybe)
    cp = np.concatenate([[0], np.cumsum([len(r) for r in rows])]).astype(np.int64)
    cc = np.concatenate([np.asarray(r, dtype=np.int32) for r in rows])
    pp, pa, pb = amg.product_plan(A.indptr, A.indices, B.indptr, B.indices, cp, cc, 25)
    for i in range(40):
        for ci in range(cp[i], cp[i + 1]):
            want = []
            for ak in range(A.indptr[i], A.indptr[i + 1]):
                k = A.indices[ak]
                for bk in range(B.indptr[k], B.indptr[k + 1]):
                    if B.indices[bk] == cc[ci]:
                        want.append((ak, bk))
            got = list(zip(pa[pp[ci]:pp[ci + 1]], pb[pp[ci]:pp[ci + 1]]))
            assert got == want, (i, ci)


def test_product_plan_threaded_rows():
    """The plan over enough rows that the library splits them across threads: every pair lands on
    its block (A row = C row, A column = B row, B column = C column), in A's row order, and every
    structural product into C's pattern is listed once."""
    rng = np.random.default_rng(5)

    def pattern(n, m, per_row):  # (scipy.sparse.random samples slowly at these sizes)
        M = sp.csr_matrix((np.ones(n * per_row), rng.integers(0, m, n * per_row),
                           np.arange(0, n * per_row + 1, per_row)), shape=(n, m))
        M.sum_duplicates()
        M.sort_indices()
        return M

    A, B = pattern(30000, 20000, 6), pattern(20000, 9000, 4)
    p, c = amg.symbolic(A.indptr, A.indices, B.indptr, B.indices, 9000)
    pp, pa, pb = amg.product_plan(A.indptr, A.indices, B.indptr, B.indices, p, c, 9000)
    a_row = np.repeat(np.arange(30000), np.diff(A.indptr))
    b_row = np.repeat(np.arange(20000), np.diff(B.indptr))
    c_row = np.repeat(np.arange(30000), np.diff(p))
    owner = np.repeat(np.arange(len(c)), np.diff(pp))
    assert np.array_equal(a_row[pa], c_row[owner])
    assert np.array_equal(A.indices[pa], b_row[pb])
    assert np.array_equal(B.indices[pb], c[owner])
    assert np.all((np.diff(pa) > 0) | (np.diff(owner) != 0))
    assert len(pa) == int((abs(A).astype(bool).astype(np.int64) @ abs(B).astype(bool).astype(np.int64)).sum())


def test_amg_rejects_bad_input():
    with pytest.raises(ValueError):
        amg.aggregate(np.array([0, 1]), np.array([5]))
    with pytest.raises(ValueError):
        amg.diag_index(np.array([0, 1, 2]), np.array([1, 1], dtype=np.int32))


# -- GPU ------------------------------------------------------------------------------------
def _dev():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch, torch.device("cuda:0")


def _rand_bsr(rng, n, m, br, bc, density, dev, diag=False):
    P = sp.random(n, m, density=density, random_state=int(rng.integers(1 << 30)), format="csr")
    if diag:
        P = (P + sp.eye(n, m)).tocsr()
    P.sort_indices()
    M = amg.Bsr(P.indptr, P.indices, br, bc, m, dev)
    v = rng.standard_normal(M.nnzb * br * bc)
    import torch
    M.vals[:len(v)] = torch.from_numpy(v).to(dev)
    return M


@pytest.mark.gpu
@pytest.mark.parametrize("br,bk,bc", [(3, 3, 6), (6, 3, 6), (6, 6, 6), (3, 3, 3)])
def test_bsr_kernels_match_numpy(br, bk, bc):
    torch, dev = _dev()
    rng = np.random.default_rng(br * 100 + bk * 10 + bc)
    A = _rand_bsr(rng, 50, 40, br, bk, 0.1, dev)
    B = _rand_bsr(rng, 40, 30, bk, bc, 0.12, dev)
    p, c = amg.symbolic(A.ptr_h, A.col_h, B.ptr_h, B.col_h, 30)
    C = amg.Bsr(p, c, br, bc, 30, dev)
    C.product(A, B)
    Ad, Bd = A.to_numpy(), B.to_numpy()
    ref = Ad @ Bd
    assert np.abs(C.to_numpy() - ref).max() <= 1e-13 * np.abs(ref).max()
    x = rng.standard_normal(30 * bc)
    y = torch.full((50 * br,), 2.0, dtype=torch.float64, device=dev)
    C.spmv(torch.from_numpy(x).to(dev), y, alpha=0.5, accumulate=True)
    torch.cuda.synchronize()
    assert np.abs(y.cpu().numpy() - (2.0 + 0.5 * ref @ x)).max() <= 1e-12 * np.abs(ref).max() * np.abs(x).max() * 10
    if (br, bc) in ((3, 6), (6, 6)):
        tp, tc, perm = amg.transpose_pattern(p, c, 30)
        T = amg.Bsr(tp, tc, bc, br, 50, dev)
        rc = fcg.lib().fcg_bsr_transpose_values(0, br, bc, C.nnzb, amg._vp(torch.from_numpy(perm).to(dev)),
                                                amg._vp(C.vals), amg._vp(T.vals), None)
        assert rc == 0
        torch.cuda.synchronize()
        assert np.array_equal(T.to_numpy(), C.to_numpy().T)


@pytest.mark.gpu
@pytest.mark.parametrize("br,bk,bc", [(3, 3, 6), (6, 3, 6), (6, 6, 6), (3, 3, 3)])
def test_planned_spgemm_equals_searching_spgemm(br, bk, bc):
    """fcg_bsr_spgemm_planned from fcg_bsr_product_plan: bit-identical to fcg_bsr_spgemm."""
    torch, dev = _dev()
    rng = np.random.default_rng(br * 7 + bk * 3 + bc)
    A = _rand_bsr(rng, 60, 45, br, bk, 0.1, dev)
    B = _rand_bsr(rng, 45, 35, bk, bc, 0.12, dev)
    p, c = amg.symbolic(A.ptr_h, A.col_h, B.ptr_h, B.col_h, 35)
    C1, C2 = amg.Bsr(p, c, br, bc, 35, dev), amg.Bsr(p, c, br, bc, 35, dev)
    C1.product(A, B)
    pp, pa, pb = amg.product_plan(A.ptr_h, A.col_h, B.ptr_h, B.col_h, p, c, 35)
    t = [torch.from_numpy(v).to(dev) for v in (pp, pa, pb)]
    assert fcg.lib().fcg_bsr_spgemm_planned(0, br, bk, bc, C2.nnzb, amg._vp(t[0]), amg._vp(t[1]),
                                            amg._vp(t[2]), amg._vp(A.vals), amg._vp(B.vals),
                                            amg._vp(C2.vals), None, None) == 0
    # the same blocks formed in a shuffled order
    C3 = amg.Bsr(p, c, br, bc, 35, dev)
    order = torch.from_numpy(rng.permutation(C3.nnzb).astype(np.int64)).to(dev)
    assert fcg.lib().fcg_bsr_spgemm_planned(0, br, bk, bc, C3.nnzb, amg._vp(t[0]), amg._vp(t[1]),
                                            amg._vp(t[2]), amg._vp(A.vals), amg._vp(B.vals),
                                            amg._vp(C3.vals), amg._vp(order), None) == 0
    torch.cuda.synchronize()
    assert torch.equal(C1.vals, C2.vals) and torch.equal(C1.vals, C3.vals)


@pytest.mark.gpu
def test_native_amg_planned_products_are_bit_identical(monkeypatch):
    """The native AMG's Galerkin products from product plans (default) and by the searching kernel
    (FCG_AMG_PLAN=0, read at fcg_amg_create): the same iterations and solution bit for bit."""
    torch, dev = _dev()
    dis, kin, load = _case("renumbered-totlag")
    dbc, fext = _loads(dis, load)
    ev = fcg.Evaluator(dis, kinematics=fcg.LINEAR, youngs=E, poisson=NU)
    f64 = dict(dtype=torch.float64, device=dev)
    K = torch.zeros(dis.nnz, **f64)
    ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, torch.zeros(dis.n_cols, **f64),
                       torch.zeros(dis.n_rows, **f64), K)
    b = torch.from_numpy(fext).to(dev)
    ev.dirichlet_apply(torch.from_numpy(dbc).to(dev), K, b)
    out = {}
    for plan in ("1", "0"):
        monkeypatch.setenv("FCG_AMG_PLAN", plan)
        solver = amg.NativeAMG(dis, ev, dbc)
        x = torch.empty_like(b)
        it, rel = solver.solve(K, b, x, 1e-10, 500)
        out[plan] = (it, rel, x.cpu().numpy())
        solver.close()
    assert out["1"][0] == out["0"][0] and out["1"][1] == out["0"][1]
    assert np.array_equal(out["1"][2], out["0"][2])
    ev.close()


@pytest.mark.gpu
@pytest.mark.parametrize("br,bk,bc", [(3, 3, 6), (6, 6, 6)])
def test_bsr_spgemm_long_rows(br, bk, bc):
    """Output rows far longer than the lanes of a row (each lane loops over many blocks)."""
    torch, dev = _dev()
    rng = np.random.default_rng(7)
    A = _rand_bsr(rng, 6, 5, br, bk, 0.6, dev)
    B = _rand_bsr(rng, 5, 300, bk, bc, 0.9, dev)
    p, c = amg.symbolic(A.ptr_h, A.col_h, B.ptr_h, B.col_h, 300)
    assert np.diff(p).max() > 260
    C = amg.Bsr(p, c, br, bc, 300, dev)
    C.product(A, B)
    ref = A.to_numpy() @ B.to_numpy()
    assert np.abs(C.to_numpy() - ref).max() <= 1e-13 * np.abs(ref).max()


@pytest.mark.gpu
@pytest.mark.parametrize("b", [3, 6])
def test_bsr_block_inverse_and_dense(b):
    torch, dev = _dev()
    rng = np.random.default_rng(b)
    n = 30
    S = sp.random(n, n, density=0.1, random_state=3)
    S = ((S + S.T) + sp.eye(n)).tocsr()
    S.sort_indices()
    A = amg.Bsr(S.indptr, S.indices, b, b, n, dev)
    v = rng.standard_normal((A.nnzb, b, b))
    diag = amg.diag_index(A.ptr_h, A.col_h)
    for i, k in enumerate(diag):
        G = rng.standard_normal((b, b))
        v[k] = G @ G.T + b * np.eye(b)
    # an empty scalar row (a vanished coarse DOF): zero across the whole block row
    v[A.ptr_h[4]:A.ptr_h[5], 2, :] = 0.0
    A.vals[:v.size] = torch.from_numpy(v.ravel()).to(dev)
    lvl = amg._DenseLevel(A, dev)
    lvl.setup_diag()
    torch.cuda.synchronize()
    vv = A.vals.cpu().numpy()[:v.size].reshape(v.shape)
    assert vv[diag[4], 2, 2] == 1.0
    Dinv = lvl.dinv.cpu().numpy().reshape(n, b, b)
    for i in range(n):
        assert np.abs(Dinv[i] @ vv[diag[i]] - np.eye(b)).max() <= 1e-11
    r = torch.from_numpy(rng.standard_normal(n * b)).to(dev)
    z = torch.ones(n * b, dtype=torch.float64, device=dev)
    lvl.apply_dinv(r, z, 0.5, accumulate=True)
    ref = 1.0 + 0.5 * np.concatenate([Dinv[i] @ r.cpu().numpy()[i * b:(i + 1) * b] for i in range(n)])
    torch.cuda.synchronize()
    assert np.abs(z.cpu().numpy() - ref).max() <= 1e-12 * np.abs(ref).max()
    D = torch.zeros((n * b, n * b), dtype=torch.float64, device=dev)
    assert fcg.lib().fcg_bsr_to_dense(0, b, n, amg._vp(A.ptr), amg._vp(A.col), amg._vp(A.vals),
                                      amg._vp(D), None) == 0
    torch.cuda.synchronize()
    assert np.array_equal(D.cpu().numpy(), A.to_numpy())


def _loads(dis, load, axis_load=2):
    """Clamp the x-min face, a total load `load` on the x-max face nodes (direction axis_load)."""
    x = dis.node_x[:, 0]
    clamp = np.nonzero(np.isclose(x, x.min()))[0]
    tip = np.nonzero(np.isclose(x, x.max()))[0]
    dbc = np.sort((dis.node_dof_row[clamp][:, None] + np.arange(3)).ravel()).astype(np.int32)
    fext = np.zeros(dis.n_rows)
    fext[dis.node_dof_row[tip] + axis_load] = load / len(tip)
    return dbc, fext


def _newton_pair(dis, kin, load, tol=1e-10, cls=None, **amg_kw):
    torch, dev = _dev()
    dbc, fext = _loads(dis, load)
    cls = cls or amg.AMG
    out = {}
    for name in ("pcg", "amg"):
        ev = fcg.Evaluator(dis, kinematics=kin, youngs=E, poisson=NU)
        solver = cls(dis, ev, dbc, **amg_kw) if name == "amg" else None
        nt = newton.StaticNewton(ev, fext, dbc, tol_res=tol * np.linalg.norm(fext), tol_inc=1e-9,
                                 lin_rtol=1e-12, linear_solver=solver)
        u = nt.solve()
        out[name] = (u.cpu().numpy(), sum(h.get("lin_iter", 0) for h in nt.history),
                     solver.describe() if solver else None)
        if solver is not None and hasattr(solver, "close"):
            solver.close()
        ev.close()
    return out


@pytest.mark.gpu
def test_hierarchy_matches_its_definition():
    torch, dev = _dev()
    dis = fcg.Discretization.renumbered(fcg.BoxMesh(fcg.HEX8, (12, 4, 4), upper=(4.0, 1.0, 1.0)), seed=5)
    dbc, fext = _loads(dis, -1e-2)
    ev = fcg.Evaluator(dis, kinematics=fcg.LINEAR, youngs=E, poisson=NU)
    f64 = dict(dtype=torch.float64, device=dev)
    K = torch.zeros(dis.nnz, **f64)
    ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, torch.zeros(dis.n_cols, **f64),
                       torch.zeros(dis.n_rows, **f64), K)
    ev.dirichlet_apply(torch.from_numpy(dbc).to(dev), K)
    solver = amg.AMG(dis, ev, dbc, coarse_max=60)
    assert len(solver.levels) >= 3
    solver._prepare(K)
    torch.cuda.synchronize()
    Kd = sp.csr_matrix((K.cpu().numpy(), dis.col_lid, dis.rowptr), shape=(dis.n_rows,) * 2).toarray()
    assert np.array_equal(solver.A0.to_numpy(), Kd)
    A = Kd
    for l, st in enumerate(solver.steps):
        lv = solver.levels[l]
        b = st.bs
        Dinv = np.zeros_like(A)
        for i in range(A.shape[0] // b):
            s = slice(i * b, (i + 1) * b)
            blk = A[s, s].copy()
            if l > 0:  # unit diagonal on empty rows, as the device setup does
                for d in range(b):
                    if not A[i * b + d].any():
                        blk[d, d] = 1.0
            Dinv[s, s] = np.linalg.inv(blk)
        T = st.T.to_numpy()
        P = st.P.to_numpy()
        Pref = T - (solver.omega / lv.lmax) * Dinv @ A @ T
        assert np.abs(P - Pref).max() <= 1e-12 * np.abs(Pref).max()
        Ac = solver.levels[l + 1].A.to_numpy()
        Acref = P.T @ A @ P
        # compare before the device's unit-diagonal fix of empty rows
        empty = ~Acref.any(axis=1)
        Acref[empty, empty] = 1.0
        assert np.abs(Ac - Acref).max() <= 1e-11 * np.abs(Acref).max()
        A = Ac
    ev.close()


def _case(case):
    if case == "renumbered-linear":
        return fcg.Discretization.renumbered(fcg.BoxMesh(fcg.HEX8, (16, 6, 6), upper=(4.0, 1.0, 1.0), jitter=0.1), seed=1), fcg.LINEAR, -1e-2
    if case == "renumbered-totlag":
        return fcg.Discretization.renumbered(fcg.BoxMesh(fcg.HEX8, (12, 4, 4), upper=(3.0, 1.0, 1.0)), seed=2), fcg.TOTLAG, -0.5
    if case == "tiled-beam":
        return tiled_input_mesh(load_fixture(FX), (3, 6, 2), jitter=0.15, seed=11), fcg.LINEAR, -1e-3
    return fcg.Discretization.renumbered(fcg.BoxMesh(fcg.HEX27, (6, 3, 3), upper=(3.0, 1.0, 1.0)), seed=3), fcg.TOTLAG, -0.5


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["renumbered-linear", "renumbered-totlag", "tiled-beam", "hex27"])
def test_newton_native_amg_matches_pcg(case):
    """The C-ABI AMG object (fcg_amg_create / fcg_amg_solve) in the Newton loop."""
    dis, kin, load = _case(case)
    out = _newton_pair(dis, kin, load, cls=amg.NativeAMG)
    (u0, it0, _), (u1, it1, lv) = out["pcg"], out["amg"]
    assert len(lv) >= 2 and all(l["lmax"] > 0 for l in lv[:-1])
    assert np.linalg.norm(u1 - u0) <= 1e-8 * np.linalg.norm(u0)
    assert it1 * 3 < it0, (it0, it1, lv)


@pytest.mark.gpu
@pytest.mark.parametrize("cls", ["AMG", "NativeAMG"])
def test_amg_reported_residual_is_the_true_one(cls):
    """The returned relative residual is |b - K x| / |b| of the returned x (not a stale scalar)."""
    torch, dev = _dev()
    dis, kin, load = _case("renumbered-linear")
    dbc, fext = _loads(dis, load)
    ev = fcg.Evaluator(dis, kinematics=fcg.LINEAR, youngs=E, poisson=NU)
    f64 = dict(dtype=torch.float64, device=dev)
    K = torch.zeros(dis.nnz, **f64)
    ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, torch.zeros(dis.n_cols, **f64),
                       torch.zeros(dis.n_rows, **f64), K)
    b = torch.from_numpy(fext).to(dev)
    ev.dirichlet_apply(torch.from_numpy(dbc).to(dev), K, b)
    solver = getattr(amg, cls)(dis, ev, dbc)
    for rtol in (1e-4, 1e-9):
        x = torch.empty_like(b)
        it, rel = solver.solve(K, b, x, rtol, 500)
        Kx = torch.empty_like(b)
        ev.spmv(K, x, Kx)
        true = float(torch.linalg.vector_norm(b - Kx) / torch.linalg.vector_norm(b))
        assert rel <= rtol and true <= 2 * rtol and abs(true - rel) <= 0.5 * rtol, (cls, rtol, it, rel, true)
    if hasattr(solver, "close"):
        solver.close()
    ev.close()


@pytest.mark.gpu
def test_native_amg_dense_coarse_and_graph(monkeypatch):
    """The coarsest level as its dense inverse (Gauss-Jordan per tangent) and the FCG iteration
    replayed from a captured HIP graph: the graph gives bit-identical iterates to eager launches,
    the exact coarse solve needs no more iterations than the block-Jacobi CG one, and all three
    reach the same solution."""
    torch, dev = _dev()
    dis, kin, load = _case("renumbered-totlag")
    dbc, fext = _loads(dis, load)
    ev = fcg.Evaluator(dis, kinematics=fcg.LINEAR, youngs=E, poisson=NU)
    f64 = dict(dtype=torch.float64, device=dev)
    K = torch.zeros(dis.nnz, **f64)
    ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, torch.zeros(dis.n_cols, **f64),
                       torch.zeros(dis.n_rows, **f64), K)
    b = torch.from_numpy(fext).to(dev)
    ev.dirichlet_apply(torch.from_numpy(dbc).to(dev), K, b)
    solver = amg.NativeAMG(dis, ev, dbc)
    runs = {}
    for name, env in (("graph", {"FCG_AMG_GRAPH": "1"}), ("eager", {}), ("cg", {"FCG_AMG_DENSE": "0"})):
        for k in ("FCG_AMG_GRAPH", "FCG_AMG_DENSE"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        before = solver.stats()["graph_launches"]
        x = torch.empty_like(b)
        it, rel = solver.solve(K, b, x, 1e-9, 500)
        st = solver.stats()
        runs[name] = (it, rel, x.cpu().numpy(), st["coarse_dense"], st["graph_launches"] - before)
    it_g, rel_g, x_g, dense_g, launches_g = runs["graph"]
    it_e, rel_e, x_e, dense_e, launches_e = runs["eager"]
    it_c, rel_c, x_c, dense_c, launches_c = runs["cg"]
    assert dense_g and dense_e and not dense_c
    assert launches_g >= it_g - 1 > 0 and launches_e == 0 and launches_c == 0
    assert it_g == it_e and rel_g == rel_e and np.array_equal(x_g, x_e)
    assert it_g <= it_c, (it_g, it_c)
    assert np.linalg.norm(x_g - x_c) <= 1e-7 * np.linalg.norm(x_c)
    solver.close()
    ev.close()


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["renumbered-totlag", "tiled-beam"])
def test_native_amg_morton_level0_matches_context_order(monkeypatch, case):
    """Level 0 renumbered in the Morton order of the node coordinates (default; the BSR copy in
    that order, vectors permuted on entry and exit) against the context's order
    (FCG_AMG_REORDER=0): the same solution to the solve tolerance, iteration counts alike, and
    fcg_amg_apply's V-cycle in the caller's order (a symmetric positive preconditioner)."""
    torch, dev = _dev()
    if case == "tiled-beam":
        dis, load = tiled_input_mesh(load_fixture(FX), (3, 6, 2), jitter=0.15, seed=11), -1e-3
    else:
        dis, _, load = _case(case)
    dbc, fext = _loads(dis, load)
    ev = fcg.Evaluator(dis, kinematics=fcg.LINEAR, youngs=E, poisson=NU)
    f64 = dict(dtype=torch.float64, device=dev)
    K = torch.zeros(dis.nnz, **f64)
    ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, torch.zeros(dis.n_cols, **f64),
                       torch.zeros(dis.n_rows, **f64), K)
    b = torch.from_numpy(fext).to(dev)
    ev.dirichlet_apply(torch.from_numpy(dbc).to(dev), K, b)
    out = {}
    for reorder in ("1", "0"):
        monkeypatch.setenv("FCG_AMG_REORDER", reorder)
        solver = amg.NativeAMG(dis, ev, dbc)
        x = torch.empty_like(b)
        it, rel = solver.solve(K, b, x, 1e-10, 500)
        # the V-cycle through fcg_amg_apply: r . M r > 0 for a random r (caller's order in and out)
        r = torch.randn(dis.n_rows, generator=torch.Generator().manual_seed(3), dtype=torch.float64).to(dev)
        r[torch.from_numpy(dbc.astype(np.int64)).to(dev)] = 0.0
        z = torch.empty_like(r)
        L = fcg.lib()
        assert L.fcg_amg_apply(solver._h, amg._vp(K), amg._vp(r), amg._vp(z), None) == 0
        torch.cuda.synchronize()
        out[reorder] = (it, rel, x.cpu().numpy(), float(torch.dot(r, z)))
        solver.close()
    (i1, r1, x1, q1), (i0, r0, x0, q0) = out["1"], out["0"]
    assert r1 <= 1e-10 and r0 <= 1e-10 and q1 > 0 and q0 > 0
    assert np.linalg.norm(x1 - x0) <= 1e-8 * np.linalg.norm(x0)
    assert abs(i1 - i0) <= max(2, 0.25 * i0), (i1, i0)
    ev.close()


@pytest.mark.gpu
def test_native_amg_rejects_bad_input():
    torch, dev = _dev()
    dis, kin, load = _case("renumbered-totlag")
    dbc, fext = _loads(dis, load)
    ev = fcg.Evaluator(dis, kinematics=kin, youngs=E, poisson=NU)
    with pytest.raises(fcg.FcgError):
        amg.NativeAMG(dis, ev, np.array([dis.n_rows + 5], dtype=np.int32))
    solver = amg.NativeAMG(dis, ev, dbc)
    K = torch.zeros(dis.nnz, dtype=torch.float64, device=dev)  # all-zero tangent: singular blocks
    b = torch.ones(dis.n_rows, dtype=torch.float64, device=dev)
    with pytest.raises(fcg.FcgError):
        solver.solve(K, b, torch.empty_like(b), 1e-8)
    solver.close()
    ev.close()


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["renumbered-linear", "renumbered-totlag", "tiled-beam", "hex27"])
def test_newton_amg_matches_pcg(case):
    if case == "renumbered-linear":
        dis, kin, load = fcg.Discretization.renumbered(fcg.BoxMesh(fcg.HEX8, (16, 6, 6), upper=(4.0, 1.0, 1.0), jitter=0.1), seed=1), fcg.LINEAR, -1e-2
    elif case == "renumbered-totlag":
        dis, kin, load = fcg.Discretization.renumbered(fcg.BoxMesh(fcg.HEX8, (12, 4, 4), upper=(3.0, 1.0, 1.0)), seed=2), fcg.TOTLAG, -0.5
    elif case == "tiled-beam":
        dis, kin, load = tiled_input_mesh(load_fixture(FX), (3, 6, 2), jitter=0.15, seed=11), fcg.LINEAR, -1e-3
    else:
        dis, kin, load = fcg.Discretization.renumbered(fcg.BoxMesh(fcg.HEX27, (6, 3, 3), upper=(3.0, 1.0, 1.0)), seed=3), fcg.TOTLAG, -0.5
    out = _newton_pair(dis, kin, load)
    (u0, it0, _), (u1, it1, lv) = out["pcg"], out["amg"]
    assert len(lv) >= 2
    assert np.linalg.norm(u1 - u0) <= 1e-8 * np.linalg.norm(u0)
    assert it1 * 3 < it0, (it0, it1, lv)
