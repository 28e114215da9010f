"""Shared helpers for the parity tests: run the CPU oracle on a BoxMesh's discretization.
TEST INFRASTRUCTURE ONLY."""

import ctypes
import importlib

import numpy as np

import oracle_lib as orc

fcg = importlib.import_module("4c_amd").fcg


def gid_maps(row_gid, col_gid):
    max_gid = int(max(row_gid.max(initial=0), col_gid.max(initial=0)))
    row_lid = np.full(max_gid + 1, -1, dtype=np.int32)
    col_lid = np.full(max_gid + 1, -1, dtype=np.int32)
    row_lid[row_gid] = np.arange(len(row_gid), dtype=np.int32)
    col_lid[col_gid] = np.arange(len(col_gid), dtype=np.int32)
    return row_lid, col_lid, max_gid


def oracle_evaluate(mesh, kinem, E, nu, u_col, want_k=True, nworkers=1, min_node_gid=0,
                    material=orc.MAT_STVK):
    """Oracle Discretization::evaluate on mesh's rank: returns (err, bad_ele, K_vals, fint).

    The oracle evaluates the rank's column elements and assembles the rows the rank owns, in the
    CSR pattern (rowptr/col_lid) and maps (row_gid/col_gid) of `mesh`.
    """
    lib = orc.load()
    row_lid, col_lid, max_gid = gid_maps(mesh.row_gid, mesh.col_gid)
    K = np.zeros(mesh.nnz) if want_k else None
    f = np.zeros(mesh.n_rows)
    csr = orc.OrcCsr()
    csr.n_rows = mesh.n_rows
    csr.rowptr = mesh.rowptr.ctypes.data_as(orc._i64p)
    csr.col_lid = mesh.col_lid.ctypes.data_as(orc._i32p)
    csr.vals = K.ctypes.data_as(orc._dp) if want_k else None
    csr.row_lid_of_gid = row_lid.ctypes.data_as(orc._i32p)
    csr.col_lid_of_gid = col_lid.ctypes.data_as(orc._i32p)
    csr.max_gid = max_gid
    ele_nodes = mesh.ele_nodes.astype(np.int64)
    # owner: the mesh rank's owned nodes are split into `nworkers` contiguous chunks (z-slabs,
    # since owned nodes are gid-ordered), each run as its own oracle "rank"; ghosts belong to none
    owned = mesh.node_dof_row >= 0
    owner = np.full(mesh.n_node, -1, dtype=np.int32)
    idx = np.nonzero(owned)[0]
    owner[idx] = (np.arange(len(idx)) * nworkers // max(len(idx), 1)).astype(np.int32)
    bad = ctypes.c_int64(-1)
    err = lib.orc_discretization_evaluate_mat(
        mesh.celltype, kinem, material, E, nu, mesh.n_ele, ele_nodes.ctypes.data_as(orc._i64p), mesh.n_node,
        np.ascontiguousarray(mesh.node_x).ctypes.data_as(orc._dp),
        mesh.node_gid.ctypes.data_as(orc._i64p), owner.ctypes.data_as(orc._i32p), min_node_gid,
        nworkers, u_col.ctypes.data_as(orc._dp), ctypes.byref(csr), f.ctypes.data_as(orc._dp),
        ctypes.byref(bad))
    return err, bad.value, K, f


def rel_err(a, b):
    nb = np.linalg.norm(b)
    return np.linalg.norm(a - b) / (nb if nb > 0 else 1.0)


def _csr(n_rows, rowptr, cols, vals, row_gid, col_gid):
    row_lid, col_lid, max_gid = gid_maps(np.asarray(row_gid), np.asarray(col_gid))
    c = orc.OrcCsr()
    c.n_rows = n_rows
    c.rowptr = rowptr.ctypes.data_as(orc._i64p)
    c.col_lid = cols.ctypes.data_as(orc._i32p)
    c.vals = vals.ctypes.data_as(orc._dp)
    c.row_lid_of_gid = row_lid.ctypes.data_as(orc._i32p)
    c.col_lid_of_gid = col_lid.ctypes.data_as(orc._i32p)
    c.max_gid = max_gid
    return c, (row_lid, col_lid)


def oracle_tsi_evaluate(mesh, g, E, nu, alpha, T0, conduct, timefac, timefac_d, u_col, v_col,
                        T_node, nworkers=1, min_node_gid=0):
    """Oracle TSI::Monolithic element loop (orc_tsi_discretization_evaluate) on a BoxMesh rank and
    its TsiGraph: returns (err, Kss, Kst, Kts, Ktt values in the graphs' CSR order, f_s, f_t).
    T_node: nodal temperatures (node order of the mesh)."""
    lib = orc.load()
    row_s, col_s = mesh.row_gid, mesh.col_gid
    # thermo maps: one DOF per node, gid = structural gid / 3 (node order kept)
    row_t, col_t = row_s[::3] // 3, col_s[::3] // 3
    vals = [np.zeros(mesh.nnz), np.zeros(g.nnz_st), np.zeros(g.nnz_ts), np.zeros(g.nnz_tt)]
    keep = []
    css, k1 = _csr(mesh.n_rows, mesh.rowptr, mesh.col_lid, vals[0], row_s, col_s)
    cst, k2 = _csr(mesh.n_rows, g.rowptr_st, g.col_st, vals[1], row_s, col_t)
    cts, k3 = _csr(g.n_rows_t, g.rowptr_ts, g.col_ts, vals[2], row_t, col_s)
    ctt, k4 = _csr(g.n_rows_t, g.rowptr_tt, g.col_tt, vals[3], row_t, col_t)
    keep += [k1, k2, k3, k4]
    T_col = np.zeros(g.n_cols_t)
    T_col[g.node_dof_col_t] = T_node
    fs, ft = np.zeros(mesh.n_rows), np.zeros(g.n_rows_t)
    owned = mesh.node_dof_row >= 0
    owner = np.full(mesh.n_node, -1, dtype=np.int32)
    idx = np.nonzero(owned)[0]
    owner[idx] = (np.arange(len(idx)) * nworkers // max(len(idx), 1)).astype(np.int32)
    en = mesh.ele_nodes.astype(np.int64)
    bad = ctypes.c_int64(-1)
    u_col = np.ascontiguousarray(u_col, dtype=np.float64)
    v_col = np.ascontiguousarray(v_col, dtype=np.float64)
    err = lib.orc_tsi_discretization_evaluate(
        mesh.celltype, E, nu, alpha, T0, conduct, timefac, timefac_d, mesh.n_ele,
        en.ctypes.data_as(orc._i64p), np.ascontiguousarray(mesh.node_x).ctypes.data_as(orc._dp),
        mesh.node_gid.ctypes.data_as(orc._i64p), owner.ctypes.data_as(orc._i32p), min_node_gid,
        nworkers, u_col.ctypes.data_as(orc._dp), v_col.ctypes.data_as(orc._dp),
        T_col.ctypes.data_as(orc._dp), ctypes.byref(css), ctypes.byref(cst), ctypes.byref(cts),
        ctypes.byref(ctt), fs.ctypes.data_as(orc._dp), ft.ctypes.data_as(orc._dp), ctypes.byref(bad))
    return (err,) + tuple(vals) + (fs, ft)


def oracle_evaluate_single(dis, kinem, E, nu, u_col, want_k=True, nworkers=1):
    """oracle_evaluate for a single-rank fcg.Discretization (DOF LID = GID, node GID = index)."""
    m = type("SingleRank", (), {})()
    m.row_gid = m.col_gid = np.arange(dis.n_cols, dtype=np.int32)
    m.nnz, m.n_rows, m.rowptr, m.col_lid = dis.nnz, dis.n_rows, dis.rowptr, dis.col_lid
    m.celltype, m.n_ele, m.ele_nodes = dis.celltype, dis.n_ele, dis.ele_nodes
    m.n_node, m.node_x, m.node_dof_row = dis.n_node, dis.node_x, dis.node_dof_row
    m.node_gid = np.arange(dis.n_node, dtype=np.int64)
    return oracle_evaluate(m, kinem, E, nu, u_col, want_k=want_k, nworkers=nworkers)


def tiled_input_mesh(fx, reps, jitter, seed):
    """A reference input mesh (fixture `fx`, hex8) tiled reps[0] x reps[1] x reps[2] times along
    its bounding box, coincident nodes merged, interior nodes jittered by `jitter` x the smallest
    edge, then node and element numbering shuffled -- an unstructured mesh that keeps the input's
    own element node orderings.  Returns an fcg.Discretization (no lattice hint)."""
    ids = sorted(int(k) for k in fx["nodes"])
    pos = {n: i for i, n in enumerate(ids)}
    X0 = np.array([fx["nodes"][str(n)] for n in ids], dtype=np.float64)
    E0 = np.array([[pos[n] for n in el["nodes"]] for el in fx["elements"] if el["shape"] == "HEX8"])
    lo, hi = X0.min(axis=0), X0.max(axis=0)
    L = hi - lo
    Xs, Es = [], []
    off = 0
    for i in range(reps[0]):
        for j in range(reps[1]):
            for k in range(reps[2]):
                Xs.append(X0 + L * np.array([i, j, k]))
                Es.append(E0 + off)
                off += len(X0)
    X = np.vstack(Xs)
    En = np.vstack(Es)
    key = np.round((X - lo) / L.max() * 2**20).astype(np.int64)
    _, first, inv = np.unique(key, axis=0, return_index=True, return_inverse=True)
    inv = inv.ravel()
    X = X[first]
    En = inv[En]
    rng = np.random.default_rng(seed)
    h = np.min([np.linalg.norm(X[En[:, a]] - X[En[:, b]], axis=1).min()
                for a, b in ((0, 1), (1, 2), (0, 4))])
    span = L * np.array(reps)
    interior = np.all((X > lo + 1e-9 * span) & (X < lo + span - 1e-9 * span), axis=1)
    X[interior] += jitter * h * rng.uniform(-1, 1, size=(interior.sum(), 3))
    perm = rng.permutation(len(X))
    newX = np.empty_like(X)
    newX[perm] = X
    En = perm[En][rng.permutation(len(En))]
    return fcg.Discretization.from_elements(fcg.HEX8, En, newX)
