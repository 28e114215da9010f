"""GPU parity: the HIP path (through the C ABI) against the CPU oracle on the same inputs.

Tolerances (BASELINE.json north_star):
  residual / internal force:  ||f_gpu - f_ref||_2 / ||f_ref||_2 <= 1e-10
  tangent:                    ||K_gpu - K_ref||_F / ||K_ref||_F <= 1e-12 and
                              max|dK| <= 1e-12 max|K_ref|
  DOF indexing / pattern:     identical CSR (same rowptr/col_lid handed to both sides), exact.
The GPU kernel uses the isotropic (lambda, mu) form of B^T C B and sums contributions
in a different order than the reference, so equality is to rounding, not bitwise; the GPU result
itself is bitwise reproducible run to run (no atomics), which is tested too.
"""

import importlib

import numpy as np
import pytest

from parity_util import oracle_evaluate, rel_err

fcg = importlib.import_module("4c_amd").fcg
torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

E, NU = 210.0, 0.3


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _run_gpu(mesh, kinem, u_col, action=fcg.CALC_NLNSTIFF, mode=fcg.OVERWRITE, ev=None,
             K0=None, f0=None, path=fcg.PATH_AUTO):
    dev = _dev()
    ev = ev or fcg.Evaluator(mesh, kinematics=kinem, youngs=E, poisson=NU, device=0, path=path)
    u = torch.from_numpy(u_col).to(dev)
    f = torch.from_numpy(f0).to(dev) if f0 is not None else torch.zeros(mesh.n_rows, dtype=torch.float64, device=dev)
    K = None
    if action == fcg.CALC_NLNSTIFF:
        K = torch.from_numpy(K0).to(dev) if K0 is not None else torch.full((mesh.nnz,), float("nan"), dtype=torch.float64, device=dev)
    ev.evaluate_device(action, mode, u, f, K)
    torch.cuda.synchronize()
    return (K.cpu().numpy() if K is not None else None), f.cpu().numpy(), ev


def _check(Kg, fg, Kr, fr):
    assert rel_err(fg, fr) <= 1e-10, rel_err(fg, fr)
    if Kg is not None:
        assert np.all(np.isfinite(Kg))
        assert rel_err(Kg, Kr) <= 1e-12, rel_err(Kg, Kr)
        assert np.abs(Kg - Kr).max() <= 1e-12 * np.abs(Kr).max()


CASES = [
    (fcg.HEX8, fcg.LINEAR, (10, 10, 10), 1e-3),
    (fcg.HEX8, fcg.TOTLAG, (6, 5, 4), 5e-2),
    (fcg.HEX27, fcg.LINEAR, (3, 3, 3), 1e-3),
    (fcg.HEX27, fcg.TOTLAG, (3, 2, 2), 5e-2),
]


@pytest.mark.parametrize("celltype,kinem,iv,amp", CASES)
def test_nlnstiff_matches_oracle(celltype, kinem, iv, amp):
    mesh = fcg.BoxMesh(celltype, iv, jitter=0.1, seed=20251015)
    u = mesh.u_col(amp)
    err, _, Kr, fr = oracle_evaluate(mesh, kinem, E, NU, u)
    assert err == 0
    Kg, fg, ev = _run_gpu(mesh, kinem, u)
    # box meshes carry the lattice hint -> hex8: fused structured sweep; hex27: general path
    # (the colour-ordered path is tested below)
    assert ev.info.path == (fcg.PATH_STRUCTURED if celltype == fcg.HEX8 else fcg.PATH_GENERAL)
    _check(Kg, fg, Kr, fr)


@pytest.mark.parametrize("kinem", [fcg.LINEAR, fcg.TOTLAG])
@pytest.mark.parametrize("iv", [(10, 10, 10), (7, 5, 9), (1, 1, 1), (13, 3, 2)])
def test_hex8_general_and_structured_paths_agree_with_oracle(kinem, iv):
    mesh = fcg.BoxMesh(fcg.HEX8, iv, jitter=0.1, seed=7)
    u = mesh.u_col(1e-3 if kinem == fcg.LINEAR else 5e-2)
    _, _, Kr, fr = oracle_evaluate(mesh, kinem, E, NU, u)
    for path in (fcg.PATH_GENERAL, fcg.PATH_STRUCTURED):
        Kg, fg, ev = _run_gpu(mesh, kinem, u, path=path)
        assert ev.info.path == path
        _check(Kg, fg, Kr, fr)


@pytest.mark.parametrize("celltype,kinem,iv,amp", CASES[:1] + CASES[3:])
def test_internal_force_only(celltype, kinem, iv, amp):
    mesh = fcg.BoxMesh(celltype, iv, jitter=0.1)
    u = mesh.u_col(amp)
    _, _, _, fr = oracle_evaluate(mesh, kinem, E, NU, u, want_k=False)
    _, fg, _ = _run_gpu(mesh, kinem, u, action=fcg.CALC_INTERNALFORCE)
    assert rel_err(fg, fr) <= 1e-10


def test_accumulate_adds_to_caller_storage():
    mesh = fcg.BoxMesh(fcg.HEX8, (4, 4, 4), jitter=0.1)
    u = mesh.u_col(1e-3)
    rng = np.random.default_rng(0)
    K0 = rng.standard_normal(mesh.nnz)
    f0 = rng.standard_normal(mesh.n_rows)
    Kg, fg, _ = _run_gpu(mesh, fcg.LINEAR, u, mode=fcg.ACCUMULATE, K0=K0.copy(), f0=f0.copy())
    Kr, fr, _ = _run_gpu(mesh, fcg.LINEAR, u, mode=fcg.OVERWRITE)
    np.testing.assert_allclose(Kg, K0 + Kr, rtol=0, atol=1e-13 * np.abs(Kr).max())
    np.testing.assert_allclose(fg, f0 + fr, rtol=0, atol=1e-13 * np.abs(fr).max())


def test_host_pointer_entry_point():
    mesh = fcg.BoxMesh(fcg.HEX27, (2, 2, 2), jitter=0.1)
    u = mesh.u_col(5e-2)
    _dev()
    ev = fcg.Evaluator(mesh, kinematics=fcg.TOTLAG, youngs=E, poisson=NU)
    K = np.zeros(mesh.nnz)
    f = np.zeros(mesh.n_rows)
    ev.evaluate(fcg.CALC_NLNSTIFF, u, f, K)
    _, _, Kr, fr = oracle_evaluate(mesh, fcg.TOTLAG, E, NU, u)
    _check(K, f, Kr, fr)


def test_bitwise_reproducible():
    mesh = fcg.BoxMesh(fcg.HEX8, (8, 8, 8), jitter=0.1)
    u = mesh.u_col(1e-3)
    K1, f1, ev = _run_gpu(mesh, fcg.LINEAR, u)
    K2, f2, _ = _run_gpu(mesh, fcg.LINEAR, u, ev=ev)
    assert np.array_equal(K1, K2) and np.array_equal(f1, f2)


def test_negative_jacobian_reports_element():
    # x -> -x turns every element inside out: det J < 0 at all nodes (calc_lib.hpp:492-494)
    mesh = fcg.BoxMesh(fcg.HEX8, (2, 2, 2))
    mesh.node_x[:, 0] *= -1.0
    with pytest.raises(fcg.FcgError) as ei:
        _run_gpu(mesh, fcg.LINEAR, np.zeros(mesh.n_cols))
    assert ei.value.code == 1
    assert ei.value.bad_ele_gid == 0  # lowest failing element gid


def test_multirank_rows_sum_to_global():
    """Ghost-layer semantics: each rank evaluates its column elements and writes owned rows; the
    union of the ranks' rows equals the single-rank assembly."""
    iv = (6, 4, 4)
    glob = fcg.BoxMesh(fcg.HEX8, iv, jitter=0.1)
    ug = glob.u_col(1e-3)
    Kg, fg, _ = _run_gpu(glob, fcg.LINEAR, ug)
    grow = {int(g): i for i, g in enumerate(glob.row_gid)}
    gcol = {int(g): i for i, g in enumerate(glob.col_gid)}
    for r in range(2):
        m = fcg.BoxMesh(fcg.HEX8, iv, jitter=0.1, rank=r, nranks=2)
        u = np.array([ug[gcol[int(g)]] for g in m.col_gid])
        K, f, _ = _run_gpu(m, fcg.LINEAR, u)
        for i in range(m.n_rows):
            gi = grow[int(m.row_gid[i])]
            assert abs(f[i] - fg[gi]) <= 1e-12 * np.abs(fg).max()
            cols = m.col_gid[m.col_lid[m.rowptr[i]:m.rowptr[i + 1]]]
            gcols = glob.col_gid[glob.col_lid[glob.rowptr[gi]:glob.rowptr[gi + 1]]]
            mine = dict(zip(cols.tolist(), K[m.rowptr[i]:m.rowptr[i + 1]].tolist()))
            ref = dict(zip(gcols.tolist(), Kg[glob.rowptr[gi]:glob.rowptr[gi + 1]].tolist()))
            assert mine.keys() == ref.keys()
            for c in mine:
                assert abs(mine[c] - ref[c]) <= 1e-12 * np.abs(Kg).max()


@pytest.mark.parametrize("celltype,kinem", [(fcg.HEX8, fcg.LINEAR), (fcg.HEX8, fcg.TOTLAG), (fcg.HEX27, fcg.TOTLAG)])
def test_more_ranks_than_elements_empty_ranks_evaluate(celltype, kinem):
    """A 2 x 1 x 1 box over 5 ranks: the ranks GridGenerator gives no elements create empty
    contexts whose evaluates (device, host, internal force, async check) are no-ops, and the other
    ranks' owned rows still equal the single-rank assembly."""
    iv, nranks = (2, 1, 1), 5
    glob = fcg.BoxMesh(celltype, iv, jitter=0.05)
    ug = glob.u_col(1e-3)
    Kg, fg, _ = _run_gpu(glob, kinem, ug)
    grow = {int(g): i for i, g in enumerate(glob.row_gid)}
    gcol = {int(g): i for i, g in enumerate(glob.col_gid)}
    empty = 0
    for r in range(nranks):
        m = fcg.BoxMesh(celltype, iv, jitter=0.05, rank=r, nranks=nranks)
        u = np.array([ug[gcol[int(g)]] for g in m.col_gid], dtype=np.float64)
        K, f, ev = _run_gpu(m, kinem, u)
        if m.n_ele == 0:
            empty += 1
            assert K.size == 0 and f.size == 0
            ev.evaluate(fcg.CALC_INTERNALFORCE, u, np.zeros(0), None)
            ev.set_async(True)
            _run_gpu(m, kinem, u, ev=ev)
            ev.check_error()
            ev.set_async(False)
        for i in range(m.n_owned_rows):
            gi = grow[int(m.row_gid[i])]
            assert abs(f[i] - fg[gi]) <= 1e-12 * np.abs(fg).max()
            cols = m.col_gid[m.col_lid[m.rowptr[i]:m.rowptr[i + 1]]]
            gcols = glob.col_gid[glob.col_lid[glob.rowptr[gi]:glob.rowptr[gi + 1]]]
            mine = dict(zip(cols.tolist(), K[m.rowptr[i]:m.rowptr[i + 1]].tolist()))
            ref = dict(zip(gcols.tolist(), Kg[glob.rowptr[gi]:glob.rowptr[gi + 1]].tolist()))
            assert mine.keys() == ref.keys()
            for c in mine:
                assert abs(mine[c] - ref[c]) <= 1e-12 * np.abs(Kg).max()
        ev.close()
    assert empty > 0


def test_random_splits_owned_rows_equal_global():
    """Seeded random boxes (1-4 elements per direction), rank counts 1-7 (empty ranks included),
    both cell types and kinematics, hex8 through each path: every rank's owned rows equal the
    single-rank assembly's rows by GID."""
    rng = np.random.default_rng(20251018)
    paths = [fcg.PATH_AUTO, fcg.PATH_GATHER, fcg.PATH_GENERAL]
    for trial in range(14):
        ct = fcg.HEX8 if trial % 3 else fcg.HEX27
        kinem = fcg.LINEAR if trial % 2 else fcg.TOTLAG
        path = paths[trial % 3] if ct == fcg.HEX8 else fcg.PATH_AUTO
        iv = tuple(int(v) for v in rng.integers(1, 5, 3))
        nranks = int(rng.integers(1, 8))
        glob = fcg.BoxMesh(ct, iv, jitter=0.05, seed=trial)
        ug = glob.u_col(1e-3)
        Kg, fg, evg = _run_gpu(glob, kinem, ug)
        evg.close()
        grow = {int(g): i for i, g in enumerate(glob.row_gid)}
        gcol = {int(g): i for i, g in enumerate(glob.col_gid)}
        tolK, tolf = 1e-12 * np.abs(Kg).max(), 1e-12 * np.abs(fg).max()
        for r in range(nranks):
            m = fcg.BoxMesh(ct, iv, jitter=0.05, seed=trial, rank=r, nranks=nranks)
            u = np.array([ug[gcol[int(g)]] for g in m.col_gid], dtype=np.float64)
            K, f, ev = _run_gpu(m, kinem, u, path=path)
            ev.close()
            for i in range(m.n_owned_rows):
                gi = grow[int(m.row_gid[i])]
                assert abs(f[i] - fg[gi]) <= tolf, (trial, iv, nranks, r, path)
                cols = m.col_gid[m.col_lid[m.rowptr[i]:m.rowptr[i + 1]]]
                gcols = glob.col_gid[glob.col_lid[glob.rowptr[gi]:glob.rowptr[gi + 1]]]
                mine = dict(zip(cols.tolist(), K[m.rowptr[i]:m.rowptr[i + 1]].tolist()))
                ref = dict(zip(gcols.tolist(), Kg[glob.rowptr[gi]:glob.rowptr[gi + 1]].tolist()))
                assert mine.keys() == ref.keys(), (trial, iv, nranks, r, path)
                assert max(abs(mine[c] - ref[c]) for c in mine) <= tolK, (trial, iv, nranks, r, path)


def test_full_size_linear_properties():
    """1M hex8 (BASELINE config 2) at full size: K u == f_int for linear kinematics (linearity),
    K symmetric by gid, and a z-slab of rows against the oracle."""
    dev = _dev()
    mesh = fcg.BoxMesh(fcg.HEX8, (100, 100, 100), jitter=0.1)
    u = mesh.u_col(1e-3)
    ev = fcg.Evaluator(mesh, kinematics=fcg.LINEAR, youngs=E, poisson=NU)
    ut = torch.from_numpy(u).to(dev)
    f = torch.zeros(mesh.n_rows, dtype=torch.float64, device=dev)
    K = torch.empty(mesh.nnz, dtype=torch.float64, device=dev)
    ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, ut, f, K)
    A = torch.sparse_csr_tensor(torch.from_numpy(mesh.rowptr).to(dev),
                                torch.from_numpy(mesh.col_lid.astype(np.int64)).to(dev), K,
                                size=(mesh.n_rows, mesh.n_cols))
    Ku = torch.mv(A, ut)
    lin = (torch.linalg.norm(Ku - f) / torch.linalg.norm(f)).item()
    assert lin <= 1e-10, lin
    del A, Ku
    # oracle on the full mesh with 16 workers (reference MPI semantics, threads as ranks)
    err, _, Kr, fr = oracle_evaluate(mesh, fcg.LINEAR, E, NU, u, nworkers=16)
    assert err == 0
    _check(K.cpu().numpy(), f.cpu().numpy(), Kr, fr)


# ------------------------------------------------------------------ ElastHyper / CoupNeoHooke
NH = fcg.MAT_ELASTHYPER_COUPNEOHOOKE


@pytest.mark.parametrize("celltype,iv", [(fcg.HEX8, (4, 3, 3)), (fcg.HEX27, (2, 2, 1))])
def test_neohooke_matches_oracle(celltype, iv):
    import oracle_lib as orc
    _dev()
    mesh = fcg.BoxMesh(celltype, iv, jitter=0.1 if celltype == fcg.HEX8 else 0.02, seed=9)
    u = mesh.u_col(5e-2)
    err, _, Kr, fr = oracle_evaluate(mesh, fcg.TOTLAG, 10.0, 0.25, u, material=orc.MAT_NEOHOOKE)
    assert err == 0
    for path in (fcg.PATH_GENERAL, fcg.PATH_COLORED):
        if path == fcg.PATH_COLORED and celltype != fcg.HEX27:
            continue
        ev = fcg.Evaluator(mesh, kinematics=fcg.TOTLAG, youngs=10.0, poisson=0.25, material=NH,
                           path=path)
        assert ev.info.path == path
        Kg, fg, _ = _run_gpu(mesh, fcg.TOTLAG, u, ev=ev)
        _check(Kg, fg, Kr, fr)
        _, fi, _ = _run_gpu(mesh, fcg.TOTLAG, u, action=fcg.CALC_INTERNALFORCE, ev=ev)
        assert rel_err(fi, fr) <= 1e-10


# ------------------------------------------------------------------ hex27 colour-ordered path
@pytest.mark.parametrize("kinem", [fcg.LINEAR, fcg.TOTLAG])
@pytest.mark.parametrize("iv", [(1, 1, 1), (2, 3, 4), (5, 1, 2), (4, 4, 4)])
def test_hex27_colored_and_general_paths_agree_with_oracle(kinem, iv):
    """Every entry of an owned row is written by the first element of the colour order that holds
    both nodes (K starts as NaN, so a missed entry shows), the others add: same K and f as the
    oracle and as the scratch + row-gather path."""
    mesh = fcg.BoxMesh(fcg.HEX27, iv, jitter=0.02, seed=11)
    u = mesh.u_col(1e-3 if kinem == fcg.LINEAR else 5e-2)
    _, _, Kr, fr = oracle_evaluate(mesh, kinem, E, NU, u)
    for path in (fcg.PATH_GENERAL, fcg.PATH_STRUCTURED):
        Kg, fg, ev = _run_gpu(mesh, kinem, u, path=path)
        assert ev.info.path == (fcg.PATH_GENERAL if path == fcg.PATH_GENERAL else fcg.PATH_COLORED)
        _check(Kg, fg, Kr, fr)
    _, fi, _ = _run_gpu(mesh, kinem, u, action=fcg.CALC_INTERNALFORCE, ev=ev)
    assert rel_err(fi, fr) <= 1e-10


def test_hex27_colored_accumulate_and_reproducible():
    mesh = fcg.BoxMesh(fcg.HEX27, (3, 3, 2), jitter=0.02)
    u = mesh.u_col(5e-2)
    rng = np.random.default_rng(1)
    K0 = rng.standard_normal(mesh.nnz)
    f0 = rng.standard_normal(mesh.n_rows)
    Ka, fa, ev = _run_gpu(mesh, fcg.TOTLAG, u, mode=fcg.ACCUMULATE, K0=K0.copy(), f0=f0.copy(),
                          path=fcg.PATH_COLORED)
    assert ev.info.path == fcg.PATH_COLORED
    K1, f1, _ = _run_gpu(mesh, fcg.TOTLAG, u, ev=ev)
    K2, f2, _ = _run_gpu(mesh, fcg.TOTLAG, u, ev=ev)
    assert np.array_equal(K1, K2) and np.array_equal(f1, f2)
    np.testing.assert_allclose(Ka, K0 + K1, rtol=0, atol=1e-13 * np.abs(K1).max())
    np.testing.assert_allclose(fa, f0 + f1, rtol=0, atol=1e-13 * np.abs(f1).max())


@pytest.mark.parametrize("nranks", [2, 3, 8])
def test_hex27_colored_multirank_rows_equal_global(nranks):
    """Box ranks (owned + ghost elements): the colour rule sees missing neighbours at the rank
    boundary only for rows the rank does not own; the union of owned rows equals the global K, f."""
    iv = (4, 3, 3)
    glob = fcg.BoxMesh(fcg.HEX27, iv, jitter=0.02)
    ug = glob.u_col(5e-2)
    Kg, fg, _ = _run_gpu(glob, fcg.TOTLAG, ug)
    grow = {int(g): i for i, g in enumerate(glob.row_gid)}
    gcol = {int(g): i for i, g in enumerate(glob.col_gid)}
    for r in range(nranks):
        m = fcg.BoxMesh(fcg.HEX27, iv, jitter=0.02, rank=r, nranks=nranks)
        u = np.array([ug[gcol[int(g)]] for g in m.col_gid])
        K, f, ev = _run_gpu(m, fcg.TOTLAG, u, path=fcg.PATH_COLORED)
        assert ev.info.path == fcg.PATH_COLORED
        gi = np.array([grow[int(g)] for g in m.row_gid])
        np.testing.assert_allclose(f, fg[gi], rtol=0, atol=1e-12 * np.abs(fg).max())
        for i in range(m.n_rows):
            cols = m.col_gid[m.col_lid[m.rowptr[i]:m.rowptr[i + 1]]]
            gcols = glob.col_gid[glob.col_lid[glob.rowptr[gi[i]]:glob.rowptr[gi[i] + 1]]]
            assert np.array_equal(np.sort(cols), np.sort(gcols))
            mine = K[m.rowptr[i]:m.rowptr[i + 1]][np.argsort(cols)]
            ref = Kg[glob.rowptr[gi[i]]:glob.rowptr[gi[i] + 1]][np.argsort(gcols)]
            np.testing.assert_allclose(mine, ref, rtol=0, atol=1e-12 * np.abs(Kg).max())


# ------------------------------------------------------------------ error paths (4C's throws)
# A hex27 element (coordinates x 1/8) whose 27 nodal Jacobian determinants are positive but whose
# Jacobian at the centre Gauss point (0, 0, 0) is exactly singular: invert3x3 throws
# "determinant of 3x3 matrix is zero" (4C_linalg_fixedsizematrix.hpp:1394) after the nodal check
# passed (calc_lib.hpp:475-496).  Found by a search over quarter-grid perturbations of the unit
# hex27 with the z-face centre difference forced into the span of the x- and y-face differences;
# every product at the centre point is exact, so det J == 0.0 on any summation order.
SINGULAR_HEX27_X4 = [  # x 1/8
    [-32, -32, -32], [36, -28, -32], [32, 32, -32], [-30, 28, -36], [-32, -32, 32], [32, -32, 32],
    [32, 32, 30], [-36, 34, 30], [0, -32, -32], [36, 4, -30], [0, 32, -32], [-32, 0, -32],
    [-26, -38, 6], [26, -38, 4], [32, 32, 0], [-32, 32, 0], [0, -32, 32], [32, 0, 32], [0, 32, 32],
    [-32, 0, 32], [0, 0, -32], [2, -36, 2], [26, 0, 2], [0, 32, 0], [-32, 0, 0], [1, -34, -31],
    [0, 0, 0]]


def _singular_hex27_mesh(n_before):
    """n_before regular hex27 elements, then the singular one (element GID n_before + 100)."""
    X = [np.array(SINGULAR_HEX27_X4, dtype=float) / 8.0]
    en = [np.arange(27)]
    for k in range(n_before):  # regular cubes, apart from each other
        X.append(4.0 * orc_par27() + 20.0 * (k + 1))
        en.append(np.arange(27) + 27 * (k + 1))
    dis = fcg.Discretization.from_elements(fcg.HEX27, np.array(en[1:] + en[:1]), np.vstack(X))
    dis.ele_gid = np.arange(100, 100 + dis.n_ele, dtype=np.int32)
    return dis


def orc_par27():
    import oracle_lib as orc
    return orc.node_param_coords(orc.HEX27)


@pytest.mark.parametrize("n_before", [0, 3])
def test_singular_gauss_point_jacobian_reports_element(n_before):
    import oracle_lib as orc
    X = np.array(SINGULAR_HEX27_X4, dtype=float) / 8.0
    assert orc.solid_evaluate(orc.HEX27, orc.LINEAR, E, NU, X, np.zeros((27, 3)))[0] == 2
    _dev()
    dis = _singular_hex27_mesh(n_before)
    for kinem in (fcg.LINEAR, fcg.TOTLAG):
        with pytest.raises(fcg.FcgError) as ei:
            _run_gpu(dis, kinem, np.zeros(dis.n_cols), path=fcg.PATH_GENERAL)
        assert ei.value.code == 2 and ei.value.bad_ele_gid == 100 + n_before


@pytest.mark.parametrize("celltype,path", [(fcg.HEX8, fcg.PATH_GENERAL), (fcg.HEX27, fcg.PATH_GENERAL),
                                           (fcg.HEX27, fcg.PATH_COLORED)])
def test_negative_nodal_jacobian_all_paths(celltype, path):
    """calc_lib.hpp:492-494 on the general and colour-ordered paths (the structured hex8 sweep is
    test_negative_jacobian_reports_element): one inverted element in the middle of a box is
    reported by its GID, and the next evaluate of a valid state succeeds again."""
    _dev()
    mesh = fcg.BoxMesh(celltype, (3, 2, 2))
    bad = 4  # element gid 4 = lattice (1, 1, 0)
    nodes = mesh.ele_nodes[list(mesh.ele_gid).index(bad)]
    good_x = mesh.node_x.copy()
    # pull the element's interior / top nodes through its bottom face (det J < 0 at its nodes)
    npe = 8 if celltype == fcg.HEX8 else 27
    top = nodes[4:8] if npe == 8 else nodes[[4, 5, 6, 7, 16, 17, 18, 19, 25]]
    mesh.node_x[top, 2] -= 1.5 * (mesh.node_x[top, 2].max() - mesh.node_x[nodes, 2].min())
    kinem = fcg.LINEAR
    # expected: the lowest GID among the elements the oracle rejects (the move also inverts
    # neighbours sharing the moved nodes); the reference throws on the first one it evaluates
    import oracle_lib as orc
    rejected = [int(g) for g, en in zip(mesh.ele_gid, mesh.ele_nodes)
                if orc.solid_evaluate(celltype, kinem, E, NU, mesh.node_x[en], np.zeros((npe, 3)),
                                      want_k=False)[0] == 1]
    assert bad in rejected
    with pytest.raises(fcg.FcgError) as ei:
        _run_gpu(mesh, kinem, np.zeros(mesh.n_cols), path=path)
    assert ei.value.code == 1 and ei.value.bad_ele_gid == min(rejected), (ei.value, rejected)
    mesh.node_x[:] = good_x
    _run_gpu(mesh, kinem, mesh.u_col(1e-3), path=path)


# ------------------------------------------------------------------ hex8 node-row gather path
def _scrambled_hex8(iv, seed, duplicate=0):
    """A jittered box turned into an 'input-file' mesh: random node numbering, random element order,
    every element's node list rotated about its local zeta axis (same orientation, different local
    numbering), no lattice hint; `duplicate` elements repeated (their nodes then belong to more
    than 8 elements, the gather's multi-chunk case)."""
    box = fcg.BoxMesh(fcg.HEX8, iv, jitter=0.1, seed=seed)
    rng = np.random.default_rng(seed)
    perm = rng.permutation(box.n_node)
    inv = np.empty_like(perm)
    inv[perm] = np.arange(box.n_node)
    X = box.node_x[perm]
    en = inv[box.ele_nodes]
    rot = rng.integers(0, 4, size=len(en))
    out = []
    for e, r in zip(en, rot):
        bot, top = list(e[:4]), list(e[4:])
        out.append(bot[r:] + bot[:r] + top[r:] + top[:r])
    out = np.array(out)
    if duplicate:
        out = np.vstack([out, out[rng.choice(len(out), duplicate, replace=False)]])
    out = out[rng.permutation(len(out))]
    return fcg.Discretization.from_elements(fcg.HEX8, out, X)


@pytest.mark.parametrize("kinem", [fcg.LINEAR, fcg.TOTLAG])
def test_renumbered_box_takes_the_sweep_by_lattice_detection(kinem):
    """An input-file-numbered box (random node and element order, no lattice hint): AUTO finds the
    lattice in the connectivity and takes the row-block sweep -- same K, f as the oracle and as the
    gather path on the same mesh; with elements' local frames rotated (4C's numbering turned about
    a local axis) the lattice is still found and K, f are unchanged."""
    _dev()
    box = fcg.BoxMesh(fcg.HEX8, (7, 6, 5), jitter=0.1, seed=12)
    dis = fcg.Discretization.renumbered(box, seed=3)
    assert dis.ele_ijk is None
    u = np.random.default_rng(2).standard_normal(dis.n_cols) * (1e-3 if kinem == fcg.LINEAR else 5e-2)
    mesh_like = type("M", (), {})()
    mesh_like.row_gid = mesh_like.col_gid = np.arange(dis.n_cols, dtype=np.int32)
    mesh_like.nnz, mesh_like.n_rows, mesh_like.rowptr, mesh_like.col_lid = dis.nnz, dis.n_rows, dis.rowptr, dis.col_lid
    mesh_like.celltype, mesh_like.n_ele, mesh_like.ele_nodes = fcg.HEX8, dis.n_ele, dis.ele_nodes
    mesh_like.n_node, mesh_like.node_x, mesh_like.node_dof_row = dis.n_node, dis.node_x, dis.node_dof_row
    mesh_like.node_gid = np.arange(dis.n_node, dtype=np.int64)
    err, _, Kr, fr = oracle_evaluate(mesh_like, kinem, E, NU, u)
    assert err == 0
    Ks, fs, ev = _run_gpu(dis, kinem, u, path=fcg.PATH_AUTO)
    assert ev.info.path == fcg.PATH_STRUCTURED
    _check(Ks, fs, Kr, fr)
    Kg, fg, ev = _run_gpu(dis, kinem, u, path=fcg.PATH_GATHER)
    assert ev.info.path == fcg.PATH_GATHER
    _check(Kg, fg, Kr, fr)
    en = dis.ele_nodes.copy()
    en[0, :4] = np.roll(en[0, :4], 1)
    en[0, 4:] = np.roll(en[0, 4:], 1)
    en[5] = en[5][[1, 5, 6, 2, 0, 4, 7, 3]]
    en[9] = en[9][[4, 7, 6, 5, 0, 3, 2, 1]]
    rot = fcg.Discretization(fcg.HEX8, en, dis.node_x, dis.node_dof_col, dis.node_dof_row,
                             dis.rowptr, dis.col_lid)
    Kt, ft, ev = _run_gpu(rot, kinem, u, path=fcg.PATH_AUTO)
    assert ev.info.path == fcg.PATH_STRUCTURED
    _check(Kt, ft, Kr, fr)


@pytest.mark.parametrize("kinem", [fcg.LINEAR, fcg.TOTLAG])
def test_sweep_deferred_lower_plane_blocks_bitwise(kinem, monkeypatch):
    """The sweep's MODE 3 (each row's lower-plane blocks written one layer later, beside the row's
    other blocks -- chosen for rows not in lattice order) stores the same values as MODE 0:
    bitwise equal K, f for OVERWRITE and ACCUMULATE on box ranks (holes at the rank faces), and on
    a renumbered box (its default for linear kinematics) the same as the oracle."""
    _dev()
    for r in range(2):
        m = fcg.BoxMesh(fcg.HEX8, (9, 7, 11), jitter=0.1, rank=r, nranks=2)
        u = m.u_col(1e-3 if kinem == fcg.LINEAR else 5e-2)
        rng = np.random.default_rng(r)
        K0, f0 = rng.standard_normal(m.nnz), rng.standard_normal(m.n_rows)
        out = {}
        for defer in ("0", "1"):
            monkeypatch.setenv("FCG_SWEEP_DEFER", defer)
            K1, f1, ev = _run_gpu(m, kinem, u, path=fcg.PATH_STRUCTURED)
            K2, f2, _ = _run_gpu(m, kinem, u, ev=ev, mode=fcg.ACCUMULATE, K0=K0, f0=f0)
            out[defer] = (K1, f1, K2, f2)
        for a, b in zip(out["0"], out["1"]):
            assert np.array_equal(a, b)
    monkeypatch.delenv("FCG_SWEEP_DEFER")
    box = fcg.BoxMesh(fcg.HEX8, (6, 7, 5), jitter=0.1, seed=8)
    dis = fcg.Discretization.renumbered(box, seed=5)
    u = np.random.default_rng(4).standard_normal(dis.n_cols) * (1e-3 if kinem == fcg.LINEAR else 5e-2)
    mesh_like = type("M", (), {})()
    mesh_like.row_gid = mesh_like.col_gid = np.arange(dis.n_cols, dtype=np.int32)
    mesh_like.nnz, mesh_like.n_rows, mesh_like.rowptr, mesh_like.col_lid = dis.nnz, dis.n_rows, dis.rowptr, dis.col_lid
    mesh_like.celltype, mesh_like.n_ele, mesh_like.ele_nodes = fcg.HEX8, dis.n_ele, dis.ele_nodes
    mesh_like.n_node, mesh_like.node_x, mesh_like.node_dof_row = dis.n_node, dis.node_x, dis.node_dof_row
    mesh_like.node_gid = np.arange(dis.n_node, dtype=np.int64)
    err, _, Kr, fr = oracle_evaluate(mesh_like, kinem, E, NU, u)
    assert err == 0
    Ks, fs, ev = _run_gpu(dis, kinem, u, path=fcg.PATH_STRUCTURED)
    _check(Ks, fs, Kr, fr)
    monkeypatch.setenv("FCG_SWEEP_DEFER", "0")
    K0s, f0s, _ = _run_gpu(dis, kinem, u, path=fcg.PATH_STRUCTURED)
    assert np.array_equal(Ks, K0s) and np.array_equal(fs, f0s)


def test_lattice_detection_with_holes_matches_oracle():
    """Lattice detection on an input-file mesh with elements missing (a hole through the box and an
    L-shaped notch): the found lattice has empty positions, which the row-block sweep treats like
    a rank's missing neighbours -- same K, f as the oracle."""
    _dev()
    box = fcg.BoxMesh(fcg.HEX8, (6, 5, 4), jitter=0.1, seed=21)
    keep = np.ones(box.n_ele, dtype=bool)
    ijk = box.ele_ijk
    keep &= ~((ijk[:, 0] == 2) & (ijk[:, 1] == 2))                    # a hole along z
    keep &= ~((ijk[:, 0] >= 4) & (ijk[:, 1] >= 3) & (ijk[:, 2] >= 2))  # a notch at a corner
    en = box.ele_nodes[keep]
    used = np.unique(en)
    renum = np.full(box.n_node, -1, dtype=np.int64)
    renum[used] = np.random.default_rng(4).permutation(len(used))
    X = np.empty((len(used), 3))
    X[renum[used]] = box.node_x[used]
    en = renum[en][np.random.default_rng(5).permutation(len(en))]
    dis = fcg.Discretization.from_elements(fcg.HEX8, en, X)
    u = np.random.default_rng(6).standard_normal(dis.n_cols) * 1e-3
    mesh_like = type("M", (), {})()
    mesh_like.row_gid = mesh_like.col_gid = np.arange(dis.n_cols, dtype=np.int32)
    mesh_like.nnz, mesh_like.n_rows, mesh_like.rowptr, mesh_like.col_lid = dis.nnz, dis.n_rows, dis.rowptr, dis.col_lid
    mesh_like.celltype, mesh_like.n_ele, mesh_like.ele_nodes = fcg.HEX8, dis.n_ele, dis.ele_nodes
    mesh_like.n_node, mesh_like.node_x, mesh_like.node_dof_row = dis.n_node, dis.node_x, dis.node_dof_row
    mesh_like.node_gid = np.arange(dis.n_node, dtype=np.int64)
    err, _, Kr, fr = oracle_evaluate(mesh_like, fcg.LINEAR, E, NU, u)
    assert err == 0
    Ks, fs, ev = _run_gpu(dis, fcg.LINEAR, u, path=fcg.PATH_AUTO)
    assert ev.info.path == fcg.PATH_STRUCTURED
    _check(Ks, fs, Kr, fr)


@pytest.mark.parametrize("kinem", [fcg.LINEAR, fcg.TOTLAG])
@pytest.mark.parametrize("iv,dup", [((6, 5, 4), 0), ((3, 3, 2), 5), ((1, 1, 1), 0)])
def test_gather_path_unstructured_matches_oracle(kinem, iv, dup):
    import oracle_lib as orc
    _dev()
    dis = _scrambled_hex8(iv, 3 + dup, duplicate=dup)
    u = np.random.default_rng(1).standard_normal(dis.n_cols) * (1e-3 if kinem == fcg.LINEAR else 5e-2)
    # the oracle on the same discretization (one rank: every node owned)
    mesh_like = type("M", (), {})()
    mesh_like.row_gid = mesh_like.col_gid = np.arange(dis.n_cols, dtype=np.int32)
    mesh_like.nnz, mesh_like.n_rows, mesh_like.rowptr, mesh_like.col_lid = dis.nnz, dis.n_rows, dis.rowptr, dis.col_lid
    mesh_like.celltype, mesh_like.n_ele, mesh_like.ele_nodes = fcg.HEX8, dis.n_ele, dis.ele_nodes
    mesh_like.n_node, mesh_like.node_x, mesh_like.node_dof_row = dis.n_node, dis.node_x, dis.node_dof_row
    mesh_like.node_gid = np.arange(dis.n_node, dtype=np.int64)
    err, _, Kr, fr = oracle_evaluate(mesh_like, kinem, E, NU, u)
    assert err == 0
    for path in (fcg.PATH_AUTO, fcg.PATH_GATHER, fcg.PATH_GENERAL):
        Kg, fg, ev = _run_gpu(dis, kinem, u, path=path)
        want = {fcg.PATH_GENERAL: fcg.PATH_GENERAL, fcg.PATH_GATHER: fcg.PATH_GATHER,
                # rotated element frames still stack as a lattice; repeated elements do not
                fcg.PATH_AUTO: fcg.PATH_GATHER if dup else fcg.PATH_STRUCTURED}[path]
        assert ev.info.path == want
        _check(Kg, fg, Kr, fr)
    _, fi, _ = _run_gpu(dis, kinem, u, action=fcg.CALC_INTERNALFORCE, path=fcg.PATH_GATHER)
    assert rel_err(fi, fr) <= 1e-10
    assert orc is not None


@pytest.mark.parametrize("kinem", [fcg.LINEAR, fcg.TOTLAG])
def test_gather_path_box_ranks_accumulate_reproducible(kinem):
    """Box ranks forced onto the gather path: owned rows equal the structured sweep's, ACCUMULATE
    adds, and two evaluations agree bit for bit."""
    for r in range(3):
        m = fcg.BoxMesh(fcg.HEX8, (7, 5, 6), jitter=0.1, rank=r, nranks=3)
        u = m.u_col(1e-3 if kinem == fcg.LINEAR else 5e-2)
        Ks, fs, _ = _run_gpu(m, kinem, u, path=fcg.PATH_STRUCTURED)
        K1, f1, ev = _run_gpu(m, kinem, u, path=fcg.PATH_GATHER)
        assert ev.info.path == fcg.PATH_GATHER
        _check(K1, f1, Ks, fs)
        K2, f2, _ = _run_gpu(m, kinem, u, ev=ev)
        assert np.array_equal(K1, K2) and np.array_equal(f1, f2)
        rng = np.random.default_rng(r)
        K0, f0 = rng.standard_normal(m.nnz), rng.standard_normal(m.n_rows)
        Ka, fa, _ = _run_gpu(m, kinem, u, mode=fcg.ACCUMULATE, K0=K0.copy(), f0=f0.copy(), ev=ev)
        np.testing.assert_allclose(Ka, K0 + K1, rtol=0, atol=1e-13 * np.abs(K1).max())
        np.testing.assert_allclose(fa, f0 + f1, rtol=0, atol=1e-13 * np.abs(f1).max())


def test_gather_path_negative_jacobian():
    _dev()
    dis = _scrambled_hex8((3, 2, 2), 9)
    dis.ele_gid = np.arange(50, 50 + dis.n_ele, dtype=np.int32)
    dis.node_x[:, 0] *= -1.0
    with pytest.raises(fcg.FcgError) as ei:
        _run_gpu(dis, fcg.LINEAR, np.zeros(dis.n_cols), path=fcg.PATH_GATHER)
    assert ei.value.code == 1 and ei.value.bad_ele_gid == 50
