"""Thermo-structure interaction (BASELINE config 5): the device blocks
k_ST, k_TS, k_TT and the residual parts f_S(T), f_T against the CPU oracle, and the reference's
monolithic TSI known answers (tsi_heatflux_monolithic.dat, tsi_heatflux_flexoutsurf_monolithic.dat)
reproduced with every element block coming from the library.

Tolerances as the structural path: ||dK||_F / ||K||_F <= 1e-12 per block, residuals 1e-10;
RESULT values at the reference's own (absolute) tolerances.
"""

import importlib
import json
import os

import numpy as np
import pytest

import oracle_lib as orc
from tsi_driver import TsiProblem

fcg = importlib.import_module("4c_amd").fcg
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

E, NU, ALPHA, T0, COND, DT = 210.0, 0.3, 1.2e-5, 293.0, 52.0, 0.5


def _graph_reference(mesh):
    """k_TT / k_ST / k_TS graphs straight from the element couplings (single rank)."""
    nb = [set() for _ in range(mesh.n_node)]
    for el in mesh.ele_nodes:
        for a in el:
            nb[a].update(int(b) for b in el)
    return nb


@pytest.mark.parametrize("celltype,iv,nranks", [(fcg.HEX8, (3, 3, 2), 1), (fcg.HEX8, (4, 3, 2), 2),
                                                (fcg.HEX27, (2, 1, 1), 1)])
def test_tsi_graph_is_the_node_graph(celltype, iv, nranks):
    m = fcg.BoxMesh(celltype, iv, rank=nranks - 1, nranks=nranks)
    g = fcg.TsiGraph(m)
    nb = _graph_reference(m)
    owned = np.nonzero(m.node_dof_row >= 0)[0]
    assert g.n_rows_t == len(owned) and g.n_cols_t == m.n_node
    for n in owned:
        tr = g.node_dof_row_t[n]
        cols_t = sorted(int(g.node_dof_col_t[b]) for b in nb[n])
        assert list(g.col_tt[g.rowptr_tt[tr]:g.rowptr_tt[tr + 1]]) == cols_t
        for d in range(3):
            r = m.node_dof_row[n] + d
            assert list(g.col_st[g.rowptr_st[r]:g.rowptr_st[r + 1]]) == cols_t
        cols_s = sorted(int(m.node_dof_col[b]) + d for b in nb[n] for d in range(3))
        assert list(g.col_ts[g.rowptr_ts[tr]:g.rowptr_ts[tr + 1]]) == cols_s


@pytest.mark.parametrize("iv,rank,nranks", [((4, 3, 5), 1, 3), ((2, 2, 2), 0, 1), ((7, 1, 1), 0, 1)])
def test_lattice_ijk_recovers_box_positions(iv, rank, nranks):
    m = fcg.BoxMesh(fcg.HEX8, iv, rank=rank, nranks=nranks)
    ijk = fcg.lattice_ijk(m.ele_nodes)
    assert np.array_equal(ijk, m.ele_ijk - m.ele_ijk.min(axis=0))
    en = m.ele_nodes.copy()
    en[len(en) // 2] = np.roll(en[len(en) // 2], 1)  # one element with a rotated node order
    assert fcg.lattice_ijk(en) is None or len(en) == 1


def test_lattice_ijk_on_reference_tsi_meshes():
    for name, n in (("tsi_heatflux_monolithic.json", (1, 1, 3)),
                    ("tsi_heatflux_flexoutsurf_monolithic.json", (2, 2, 3))):
        prob = TsiProblem(json.load(open(os.path.join(GOLD, name))))
        ijk = fcg.lattice_ijk(prob.elements)
        assert ijk is not None and tuple(ijk.max(axis=0) + 1) == n


def test_tsi_create_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by the gpu tests")
    m = fcg.BoxMesh(fcg.HEX8, (2, 2, 2))
    with pytest.raises(fcg.FcgError) as ei:
        fcg.TsiEvaluator(m, E, NU, ALPHA, T0, COND)
    assert ei.value.code == 4  # FCG_ERR_DEVICE


def test_tsi_invalid_material_rejected():
    m = fcg.BoxMesh(fcg.HEX8, (1, 1, 1))
    with pytest.raises(fcg.FcgError) as ei:
        fcg.TsiEvaluator(m, E, 0.5, ALPHA, T0, COND)
    assert ei.value.code == 3


# ------------------------------------------------------------------------------------ GPU
def _dev():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch, torch.device("cuda:0")


def _fields(mesh, seed=11):
    """Displacement, velocity and temperature states (column maps) of a box rank."""
    X = mesh.node_x
    u = mesh.u_col(1e-3)
    rng = np.random.default_rng(seed)
    v = 1e-2 * rng.standard_normal(mesh.n_cols)
    Tn = T0 + 50.0 * np.sin(2 * np.pi * X[:, 0]) * np.cos(np.pi * X[:, 1]) + 10.0 * X[:, 2]
    return u, v, Tn


def _oracle_blocks(mesh, g, u, v, Tn):
    """Dense (owned rows x column map) oracle blocks and residuals of the rank's column elements."""
    m = orc.st_modulus(E, NU, ALPHA)
    ns, nt = mesh.n_rows, g.n_rows_t
    Kss = np.zeros((ns, mesh.n_cols))
    Kst = np.zeros((ns, g.n_cols_t))
    Kts = np.zeros((nt, mesh.n_cols))
    Ktt = np.zeros((nt, g.n_cols_t))
    fs, fT = np.zeros(ns), np.zeros(nt)
    for en in mesh.ele_nodes:
        sc = (mesh.node_dof_col[en][:, None] + np.arange(3)).ravel()
        tc = g.node_dof_col_t[en]
        Xe, Te = mesh.node_x[en], Tn[en]
        err, Ke, fe, Kste = orc.tsi_solid_evaluate(mesh.celltype, E, NU, ALPHA, T0, Xe, u[sc], Te)
        assert err == 0
        err, Ktte, fTe, Ktse = orc.tsi_thermo_evaluate(mesh.celltype, COND, m, Xe, Te, v[sc], 1.0,
                                                       1.0 / DT)
        assert err == 0
        rows_s = (np.repeat(mesh.node_dof_row[en], 3) + np.tile(np.arange(3), len(en)))
        own_s = np.repeat(mesh.node_dof_row[en] >= 0, 3)
        rows_t = g.node_dof_row_t[en]
        own_t = rows_t >= 0
        Kss[np.ix_(rows_s[own_s], sc)] += Ke[own_s]
        Kst[np.ix_(rows_s[own_s], tc)] += Kste[own_s]
        fs[rows_s[own_s]] += fe[own_s]
        Ktt[np.ix_(rows_t[own_t], tc)] += Ktte[own_t]
        Kts[np.ix_(rows_t[own_t], sc)] += Ktse[own_t]
        fT[rows_t[own_t]] += fTe[own_t]
    return Kss, Kst, Kts, Ktt, fs, fT


def _csr_vals(D, rowptr, cols):
    rows = np.repeat(np.arange(len(rowptr) - 1), np.diff(rowptr))
    return D[rows, cols]


def _rel(a, b):
    nb = np.linalg.norm(b)
    return np.linalg.norm(a - b) / (nb if nb > 0 else 1.0)


def _gpu_all(mesh, tev, ev, u, v, Tn, mode=None, init=None):
    torch, dev = _dev()
    g = tev.graph
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).to(dev)
    fs = torch.zeros(mesh.n_rows, dtype=torch.float64, device=dev)
    Kss = torch.zeros(mesh.nnz, dtype=torch.float64, device=dev)
    ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, t(u), fs, Kss)
    out = {k: torch.full((n,), float("nan"), dtype=torch.float64, device=dev)
           for k, n in (("Kst", g.nnz_st), ("Kts", g.nnz_ts), ("Ktt", g.nnz_tt), ("fT", g.n_rows_t))}
    if init is not None:
        for k in out:
            out[k] = t(init[k])
    tev.evaluate_device(fcg.TSI_ALL, fcg.OVERWRITE if mode is None else mode, t(v), t(Tn), 1.0,
                        1.0 / DT, fs=fs, **out)
    torch.cuda.synchronize()
    res = {k: x.cpu().numpy() for k, x in out.items()}
    res["Kss"], res["fs"] = Kss.cpu().numpy(), fs.cpu().numpy()
    return res


@pytest.mark.gpu
@pytest.mark.parametrize("celltype,iv", [(fcg.HEX8, (5, 4, 3)), (fcg.HEX27, (2, 2, 1))])
def test_tsi_blocks_match_oracle(celltype, iv):
    _dev()
    mesh = fcg.BoxMesh(celltype, iv, jitter=0.1 if celltype == fcg.HEX8 else 0.02, seed=3)
    u, v, Tn = _fields(mesh)
    ev = fcg.Evaluator(mesh, kinematics=fcg.LINEAR, youngs=E, poisson=NU)
    tev = fcg.TsiEvaluator(mesh, E, NU, ALPHA, T0, COND)
    g = tev.graph
    r = _gpu_all(mesh, tev, ev, u, v, Tn)
    Kss, Kst, Kts, Ktt, fs, fT = _oracle_blocks(mesh, g, u, v, Tn)
    assert _rel(r["Kss"], _csr_vals(Kss, mesh.rowptr, mesh.col_lid)) <= 1e-12
    for name, D, rp, cl in (("Kst", Kst, g.rowptr_st, g.col_st), ("Kts", Kts, g.rowptr_ts, g.col_ts),
                            ("Ktt", Ktt, g.rowptr_tt, g.col_tt)):
        ref = _csr_vals(D, rp, cl)
        assert np.all(np.isfinite(r[name])), name
        assert _rel(r[name], ref) <= 1e-12, (name, _rel(r[name], ref))
        assert np.abs(r[name] - ref).max() <= 1e-12 * np.abs(ref).max(), name
    assert _rel(r["fs"], fs) <= 1e-10, _rel(r["fs"], fs)
    assert _rel(r["fT"], fT) <= 1e-10, _rel(r["fT"], fT)


@pytest.mark.gpu
def test_tsi_accumulate_and_reproducible():
    _dev()
    mesh = fcg.BoxMesh(fcg.HEX8, (4, 4, 3), jitter=0.1)
    u, v, Tn = _fields(mesh)
    ev = fcg.Evaluator(mesh, kinematics=fcg.LINEAR, youngs=E, poisson=NU)
    tev = fcg.TsiEvaluator(mesh, E, NU, ALPHA, T0, COND)
    g = tev.graph
    a = _gpu_all(mesh, tev, ev, u, v, Tn)
    b = _gpu_all(mesh, tev, ev, u, v, Tn)
    for k in a:
        assert np.array_equal(a[k], b[k]), k
    rng = np.random.default_rng(1)
    init = {"Kst": rng.standard_normal(g.nnz_st), "Kts": rng.standard_normal(g.nnz_ts),
            "Ktt": rng.standard_normal(g.nnz_tt), "fT": rng.standard_normal(g.n_rows_t)}
    c = _gpu_all(mesh, tev, ev, u, v, Tn, mode=fcg.ACCUMULATE, init=init)
    for k in init:
        np.testing.assert_allclose(c[k], init[k] + a[k], rtol=0, atol=1e-12 * np.abs(a[k]).max())


@pytest.mark.gpu
def test_tsi_multirank_rows_equal_global():
    """Ghost-layer semantics for the TSI blocks: each rank's owned rows equal the global rows."""
    _dev()
    iv = (6, 3, 3)
    glob = fcg.BoxMesh(fcg.HEX8, iv, jitter=0.1)
    ug, vg, Tg = _fields(glob)
    ra = _gpu_all(glob, fcg.TsiEvaluator(glob, E, NU, ALPHA, T0, COND),
                  fcg.Evaluator(glob, kinematics=fcg.LINEAR, youngs=E, poisson=NU), ug, vg, Tg)
    gg = fcg.TsiGraph(glob)
    gnode = {int(x): i for i, x in enumerate(glob.node_gid)}
    for rank in range(2):
        m = fcg.BoxMesh(fcg.HEX8, iv, jitter=0.1, rank=rank, nranks=2)
        gi = np.array([gnode[int(x)] for x in m.node_gid])
        u = np.zeros(m.n_cols)
        v = np.zeros(m.n_cols)
        for d in range(3):
            u[m.node_dof_col + d] = ug[glob.node_dof_col[gi] + d]
            v[m.node_dof_col + d] = vg[glob.node_dof_col[gi] + d]
        r = _gpu_all(m, fcg.TsiEvaluator(m, E, NU, ALPHA, T0, COND),
                     fcg.Evaluator(m, kinematics=fcg.LINEAR, youngs=E, poisson=NU), u, v, Tg[gi])
        g = fcg.TsiGraph(m)
        for n in np.nonzero(m.node_dof_row >= 0)[0]:
            G = gi[n]
            tr, gtr = g.node_dof_row_t[n], gg.node_dof_row_t[G]
            assert abs(r["fT"][tr] - ra["fT"][gtr]) <= 1e-12 * np.abs(ra["fT"]).max()
            mine = dict(zip(m.node_gid[g.col_tt[g.rowptr_tt[tr]:g.rowptr_tt[tr + 1]]].tolist(),
                            r["Ktt"][g.rowptr_tt[tr]:g.rowptr_tt[tr + 1]]))
            ref = dict(zip(glob.node_gid[gg.col_tt[gg.rowptr_tt[gtr]:gg.rowptr_tt[gtr + 1]]].tolist(),
                           ra["Ktt"][gg.rowptr_tt[gtr]:gg.rowptr_tt[gtr + 1]]))
            assert mine.keys() == ref.keys()
            for c in mine:
                assert abs(mine[c] - ref[c]) <= 1e-12 * np.abs(ra["Ktt"]).max()
            for d in range(3):
                row, grow = m.node_dof_row[n] + d, glob.node_dof_row[G] + d
                assert abs(r["fs"][row] - ra["fs"][grow]) <= 1e-12 * np.abs(ra["fs"]).max()
                a = dict(zip(m.node_gid[g.col_st[g.rowptr_st[row]:g.rowptr_st[row + 1]]].tolist(),
                             r["Kst"][g.rowptr_st[row]:g.rowptr_st[row + 1]]))
                b = dict(zip(glob.node_gid[gg.col_st[gg.rowptr_st[grow]:gg.rowptr_st[grow + 1]]].tolist(),
                             ra["Kst"][gg.rowptr_st[grow]:gg.rowptr_st[grow + 1]]))
                assert a.keys() == b.keys()
                for c in a:
                    assert abs(a[c] - b[c]) <= 1e-12 * np.abs(ra["Kst"]).max()


def _library_assembler(prob, fused=False):
    """tsi_driver assemble callback with every block from the device library (fused: one
    structured sweep pass, fcg_tsi_evaluate_fused)."""
    torch, dev = _dev()
    dis = fcg.Discretization.from_elements(prob.celltype, prob.elements, prob.X, lattice=fused)
    if fused:
        assert dis.ele_ijk is not None, "reference mesh is not a lattice"
    ev = fcg.Evaluator(dis, kinematics=fcg.LINEAR, youngs=prob.E, poisson=prob.nu,
                       path=fcg.PATH_STRUCTURED if fused else fcg.PATH_AUTO)
    tev = fcg.TsiEvaluator(dis, prob.E, prob.nu, prob.alpha, prob.T0, prob.conduct)
    g = tev.graph

    def dense(vals, rp, cl, shape):
        D = np.zeros(shape)
        rows = np.repeat(np.arange(len(rp) - 1), np.diff(rp))
        D[rows, cl] = vals
        return D

    def assemble(d, T, v):
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).to(dev)
        fs = torch.zeros(dis.n_rows, dtype=torch.float64, device=dev)
        Kss = torch.zeros(dis.nnz, dtype=torch.float64, device=dev)
        o = {k: torch.zeros(n, dtype=torch.float64, device=dev)
             for k, n in (("Kst", g.nnz_st), ("Kts", g.nnz_ts), ("Ktt", g.nnz_tt), ("fT", g.n_rows_t))}
        if fused:
            tev.evaluate_fused(ev, fcg.OVERWRITE, t(d), t(v), t(T), 1.0, 1.0 / prob.dt, fs=fs,
                               Kss=Kss, **o)
        else:
            ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, t(d), fs, Kss)
            tev.evaluate_device(fcg.TSI_ALL, fcg.OVERWRITE, t(v), t(T), 1.0, 1.0 / prob.dt, fs=fs, **o)
        o = {k: x.cpu().numpy() for k, x in o.items()}
        ns, nn = prob.ns, prob.nn
        return (dense(Kss.cpu().numpy(), dis.rowptr, dis.col_lid, (ns, ns)),
                dense(o["Kst"], g.rowptr_st, g.col_st, (ns, nn)),
                dense(o["Kts"], g.rowptr_ts, g.col_ts, (nn, ns)),
                dense(o["Ktt"], g.rowptr_tt, g.col_tt, (nn, nn)), fs.cpu().numpy(), o["fT"])
    return assemble


@pytest.mark.gpu
@pytest.mark.parametrize("fused", [False, True])
@pytest.mark.parametrize("name", ["tsi_heatflux_monolithic.json",
                                  "tsi_heatflux_flexoutsurf_monolithic.json"])
def test_tsi_result_description_on_device(name, fused):
    _dev()
    fx = json.load(open(os.path.join(GOLD, name)))
    prob = TsiProblem(fx)
    d, T = prob.solve(assemble=_library_assembler(prob, fused=fused))
    for r in fx["results"]:
        got = prob.result(d, T, r)
        assert abs(got - r["value"]) <= r["tol"], (r, got)


# ------------------------------------------------------------- fused structured sweep (config 5)
def _gpu_fused(mesh, tev, ev, u, v, Tn, mode=fcg.OVERWRITE, init=None):
    torch, dev = _dev()
    g = tev.graph
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).to(dev)
    out = {k: torch.full((n,), float("nan"), dtype=torch.float64, device=dev)
           for k, n in (("Kss", mesh.nnz), ("fs", mesh.n_rows), ("Kst", g.nnz_st),
                        ("Kts", g.nnz_ts), ("Ktt", g.nnz_tt), ("fT", g.n_rows_t))}
    if init is not None:
        for k in out:
            out[k] = t(init[k])
    tev.evaluate_fused(ev, mode, t(u), t(v), t(Tn), 1.0, 1.0 / DT, **out)
    torch.cuda.synchronize()
    return {k: x.cpu().numpy() for k, x in out.items()}


@pytest.mark.gpu
@pytest.mark.parametrize("iv,rank,nranks,jitter", [((5, 4, 3), 0, 1, 0.1), ((9, 6, 5), 0, 1, 0.0),
                                                    ((6, 5, 4), 1, 2, 0.1), ((8, 8, 8), 5, 8, 0.05)])
def test_tsi_fused_matches_oracle_and_separate_path(iv, rank, nranks, jitter):
    _dev()
    mesh = fcg.BoxMesh(fcg.HEX8, iv, jitter=jitter, seed=3, rank=rank, nranks=nranks)
    u, v, Tn = _fields(mesh)
    ev = fcg.Evaluator(mesh, kinematics=fcg.LINEAR, youngs=E, poisson=NU, path=fcg.PATH_STRUCTURED)
    tev = fcg.TsiEvaluator(mesh, E, NU, ALPHA, T0, COND)
    g = tev.graph
    r = _gpu_fused(mesh, tev, ev, u, v, Tn)
    for k, x in r.items():
        assert np.all(np.isfinite(x)), k
    Kss, Kst, Kts, Ktt, fs, fT = _oracle_blocks(mesh, g, u, v, Tn)
    for name, D, rp, cl in (("Kss", Kss, mesh.rowptr, mesh.col_lid),
                            ("Kst", Kst, g.rowptr_st, g.col_st), ("Kts", Kts, g.rowptr_ts, g.col_ts),
                            ("Ktt", Ktt, g.rowptr_tt, g.col_tt)):
        ref = _csr_vals(D, rp, cl)
        assert _rel(r[name], ref) <= 1e-12, (name, _rel(r[name], ref))
        assert np.abs(r[name] - ref).max() <= 1e-12 * np.abs(ref).max(), name
    assert _rel(r["fs"], fs) <= 1e-10, _rel(r["fs"], fs)
    assert _rel(r["fT"], fT) <= 1e-10, _rel(r["fT"], fT)
    # the two-kernel device path gives the same numbers (to rounding)
    sep = _gpu_all(mesh, tev, ev, u, v, Tn)
    for k in r:
        tol = 1e-11 if k in ("fs", "fT") else 1e-13
        assert np.abs(r[k] - sep[k]).max() <= tol * max(np.abs(sep[k]).max(), 1e-300), k


@pytest.mark.gpu
def test_tsi_fused_accumulate_and_reproducible():
    _dev()
    mesh = fcg.BoxMesh(fcg.HEX8, (6, 5, 4), jitter=0.1)
    u, v, Tn = _fields(mesh)
    ev = fcg.Evaluator(mesh, kinematics=fcg.LINEAR, youngs=E, poisson=NU, path=fcg.PATH_STRUCTURED)
    tev = fcg.TsiEvaluator(mesh, E, NU, ALPHA, T0, COND)
    a = _gpu_fused(mesh, tev, ev, u, v, Tn)
    b = _gpu_fused(mesh, tev, ev, u, v, Tn)
    for k in a:
        assert np.array_equal(a[k], b[k]), k
    rng = np.random.default_rng(2)
    init = {k: rng.standard_normal(len(x)) for k, x in a.items()}
    c = _gpu_fused(mesh, tev, ev, u, v, Tn, mode=fcg.ACCUMULATE, init=init)
    for k in init:
        np.testing.assert_allclose(c[k], init[k] + a[k], rtol=0, atol=1e-12 * np.abs(a[k]).max())


@pytest.mark.gpu
def test_tsi_fused_rejects_unqualified_contexts():
    _dev()
    mesh = fcg.BoxMesh(fcg.HEX8, (3, 3, 3))
    u, v, Tn = _fields(mesh)
    tev = fcg.TsiEvaluator(mesh, E, NU, ALPHA, T0, COND)
    for ev in (fcg.Evaluator(mesh, kinematics=fcg.LINEAR, youngs=E, poisson=NU, path=fcg.PATH_GENERAL),
               fcg.Evaluator(mesh, kinematics=fcg.TOTLAG, youngs=E, poisson=NU),
               fcg.Evaluator(mesh, kinematics=fcg.LINEAR, youngs=2 * E, poisson=NU)):
        with pytest.raises(fcg.FcgError) as ei:
            _gpu_fused(mesh, tev, ev, u, v, Tn)
        assert ei.value.code == 3
    # a structural context of another mesh fails the device identity check
    other = fcg.BoxMesh(fcg.HEX8, (3, 3, 3), jitter=0.1)
    ev = fcg.Evaluator(other, kinematics=fcg.LINEAR, youngs=E, poisson=NU, path=fcg.PATH_STRUCTURED)
    with pytest.raises(fcg.FcgError) as ei:
        _gpu_fused(mesh, tev, ev, u, v, Tn)
    assert ei.value.code == 3 and "do not share" in str(ei.value)
    hex27 = fcg.BoxMesh(fcg.HEX27, (1, 1, 1))
    with pytest.raises(fcg.FcgError) as ei:
        _gpu_fused(hex27, fcg.TsiEvaluator(hex27, E, NU, ALPHA, T0, COND),
                   fcg.Evaluator(hex27, kinematics=fcg.LINEAR, youngs=E, poisson=NU),
                   *_fields(hex27))
    assert ei.value.code == 3


@pytest.mark.gpu
@pytest.mark.parametrize("n", [100, 126])
def test_tsi_fused_full_size_properties(n):
    """Config 5's box at 100^3 and at its stated 126^3 (2M hex8): fused and two-kernel paths
    agree; f_T = K_TT T and f_S = K_SS u + K_ST (T - T_0) hold through the library's SpMV."""
    torch, dev = _dev()
    mesh = fcg.BoxMesh(fcg.HEX8, (n, n, n))
    u, v, Tn = _fields(mesh)
    ev = fcg.Evaluator(mesh, kinematics=fcg.LINEAR, youngs=E, poisson=NU, path=fcg.PATH_STRUCTURED)
    tev = fcg.TsiEvaluator(mesh, E, NU, ALPHA, T0, COND)
    g = tev.graph
    r = _gpu_fused(mesh, tev, ev, u, v, Tn)
    sep = _gpu_all(mesh, tev, ev, u, v, Tn)
    for k in r:
        # residuals: the fused pass sums f_T = K_TT T (T ~ 300 against rows summing to ~0), the
        # two-kernel path k grad T -- equal to the residual tolerance, not to the last bits
        tol = 1e-11 if k in ("fs", "fT") else 1e-13
        assert np.abs(r[k] - sep[k]).max() <= tol * np.abs(sep[k]).max(), k
    # CSR products on the host (scipy) for the size-independent identities
    sp = pytest.importorskip("scipy.sparse")
    Ktt = sp.csr_matrix((r["Ktt"], g.col_tt, g.rowptr_tt), shape=(g.n_rows_t, g.n_cols_t))
    Kss = sp.csr_matrix((r["Kss"], mesh.col_lid, mesh.rowptr), shape=(mesh.n_rows, mesh.n_cols))
    Kst = sp.csr_matrix((r["Kst"], g.col_st, g.rowptr_st), shape=(mesh.n_rows, g.n_cols_t))
    assert _rel(Ktt @ Tn, r["fT"]) <= 1e-12
    assert _rel(Kss @ u + Kst @ (Tn - T0), r["fs"]) <= 1e-12



def _fields_xyz(mesh):
    """States as functions of the node position only, so that every rank split sees the same."""
    X = mesh.node_x
    u = mesh.u_col(1e-3)
    vn = 1e-2 * np.stack([np.cos(3 * X[:, 0] + X[:, 1]), np.sin(2 * X[:, 1] - X[:, 2]),
                          np.cos(X[:, 0] * X[:, 2])], axis=1)
    v = np.zeros(mesh.n_cols)
    for d in range(3):
        v[mesh.node_dof_col + d] = vn[:, d]
    Tn = T0 + 50.0 * np.sin(2 * np.pi * X[:, 0]) * np.cos(np.pi * X[:, 1]) + 10.0 * X[:, 2]
    return u, v, Tn


@pytest.mark.gpu
def test_tsi_config5_eight_rank_split_full_size():
    """Config 5 as it is partitioned on 8 GPUs (126^3 hex8, GridGenerator split into 8 ranks with
    ghost layers), every rank evaluated in turn on one GPU: each rank's rows satisfy
    f_T = K_TT T and f_S = K_SS u + K_ST (T - T_0) on its column map, and its owned residual rows
    equal the 1-rank evaluation's by DOF / node GID."""
    torch, dev = _dev()
    sp = pytest.importorskip("scipy.sparse")
    n = 126

    from parity_util import oracle_tsi_evaluate

    def run(rank, nranks):
        mesh = fcg.BoxMesh(fcg.HEX8, (n, n, n), rank=rank, nranks=nranks)
        u, v, Tn = _fields_xyz(mesh)
        ev = fcg.Evaluator(mesh, kinematics=fcg.LINEAR, youngs=E, poisson=NU, path=fcg.PATH_STRUCTURED)
        tev = fcg.TsiEvaluator(mesh, E, NU, ALPHA, T0, COND)
        g = tev.graph
        r = _gpu_fused(mesh, tev, ev, u, v, Tn)
        ev.close()
        tev.close()
        if nranks > 1:
            # the rank's four blocks and residual rows against the oracle's TSI::Monolithic loop on
            # the same rank (its column elements, its owned rows; 16 workers)
            err, *ref = oracle_tsi_evaluate(mesh, g, E, NU, ALPHA, T0, COND, 1.0, 1.0 / DT, u, v, Tn,
                                            nworkers=16)
            assert err == 0
            for k, x in zip(("Kss", "Kst", "Kts", "Ktt", "fs", "fT"), ref):
                tol = 1e-10 if k in ("fs", "fT") else 1e-12
                assert _rel(r[k], x) <= tol, (rank, k, _rel(r[k], x))
        Ktt = sp.csr_matrix((r["Ktt"], g.col_tt, g.rowptr_tt), shape=(g.n_rows_t, g.n_cols_t))
        Kss = sp.csr_matrix((r["Kss"], mesh.col_lid, mesh.rowptr), shape=(mesh.n_rows, mesh.n_cols))
        Kst = sp.csr_matrix((r["Kst"], g.col_st, g.rowptr_st), shape=(mesh.n_rows, g.n_cols_t))
        assert _rel(Ktt @ Tn, r["fT"]) <= 1e-12, rank
        assert _rel(Kss @ u + Kst @ (Tn - T0), r["fs"]) <= 1e-12, rank
        # owned residual rows by GID (thermo row t = the node of structural rows 3t..3t+2)
        return mesh.row_gid.astype(np.int64), r["fs"], mesh.row_gid[0::3].astype(np.int64), r["fT"], \
            mesh.n_ele_global

    gs, fs1, gt, fT1, n_glob = run(0, 1)
    size = int(gs.max()) + 1
    S1, S8 = np.full(size, np.nan), np.full(size, np.nan)
    T1, T8 = np.full(size, np.nan), np.full(size, np.nan)
    S1[gs], T1[gt] = fs1, fT1
    for rank in range(8):
        a, fa, b, fb, ng = run(rank, 8)
        assert ng == n_glob == 2_000_376
        assert np.all(np.isnan(S8[a]))  # every row owned by exactly one rank
        S8[a], T8[b] = fa, fb
    assert np.array_equal(np.isnan(S1), np.isnan(S8)) and np.array_equal(np.isnan(T1), np.isnan(T8))
    ok_s, ok_t = ~np.isnan(S1), ~np.isnan(T1)
    assert np.linalg.norm(S8[ok_s] - S1[ok_s]) <= 1e-12 * np.linalg.norm(S1[ok_s])
    assert np.linalg.norm(T8[ok_t] - T1[ok_t]) <= 1e-12 * np.linalg.norm(T1[ok_t])


@pytest.mark.gpu
def test_tsi_config5_full_size_against_oracle():
    """Config 5's 126^3 box (2M hex8) at its stated size, one rank: the fused pass's four blocks
    (K_SS, k_ST, k_TS, k_TT) and both residuals against the oracle's TSI::Monolithic element loop
    on the whole mesh (orc_tsi_discretization_evaluate, 16 workers): 1e-12 / 1e-10."""
    torch, dev = _dev()
    from parity_util import oracle_tsi_evaluate
    n = 126
    mesh = fcg.BoxMesh(fcg.HEX8, (n, n, n), jitter=0.1, seed=20251015)
    u, v, Tn = _fields_xyz(mesh)
    ev = fcg.Evaluator(mesh, kinematics=fcg.LINEAR, youngs=E, poisson=NU, path=fcg.PATH_STRUCTURED)
    tev = fcg.TsiEvaluator(mesh, E, NU, ALPHA, T0, COND)
    g = tev.graph
    r = _gpu_fused(mesh, tev, ev, u, v, Tn)
    ev.close()
    tev.close()
    err, *ref = oracle_tsi_evaluate(mesh, g, E, NU, ALPHA, T0, COND, 1.0, 1.0 / DT, u, v, Tn, nworkers=16)
    assert err == 0 and mesh.n_ele == 2_000_376
    for k, x in zip(("Kss", "Kst", "Kts", "Ktt", "fs", "fT"), ref):
        tol = 1e-10 if k in ("fs", "fT") else 1e-12
        assert np.all(np.isfinite(r[k])), k
        assert _rel(r[k], x) <= tol, (k, _rel(r[k], x))
        if tol == 1e-12:
            assert np.abs(r[k] - x).max() <= 1e-12 * np.abs(x).max(), k


@pytest.mark.parametrize("nranks,nworkers", [(1, 1), (1, 4), (2, 3)])
def test_oracle_tsi_discretization_loop(nranks, nworkers):
    """orc_tsi_discretization_evaluate (the C loop the TSI CPU baseline times) equals the
    per-element Python assembly of the same oracle element routines."""
    from parity_util import oracle_tsi_evaluate
    for r in range(nranks):
        mesh = fcg.BoxMesh(fcg.HEX8, (4, 3, 3), jitter=0.1, rank=r, nranks=nranks)
        g = fcg.TsiGraph(mesh)
        u, v, Tn = _fields(mesh)
        ref = _oracle_blocks(mesh, g, u, v, Tn)
        err, Kss, Kst, Kts, Ktt, fs, fT = oracle_tsi_evaluate(mesh, g, E, NU, ALPHA, T0, COND, 1.0,
                                                              1.0 / DT, u, v, Tn, nworkers=nworkers)
        assert err == 0
        for got, (D, rp, cl) in zip((Kss, Kst, Kts, Ktt),
                                    ((ref[0], mesh.rowptr, mesh.col_lid), (ref[1], g.rowptr_st, g.col_st),
                                     (ref[2], g.rowptr_ts, g.col_ts), (ref[3], g.rowptr_tt, g.col_tt))):
            assert _rel(got, _csr_vals(D, rp, cl)) <= 1e-13
        assert _rel(fs, ref[4]) <= 1e-13 and _rel(fT, ref[5]) <= 1e-13
