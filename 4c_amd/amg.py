"""Smoothed-aggregation AMG preconditioner for the Newton solve on any single-rank mesh (SURVEY §8f
row 2 beyond GridGenerator boxes; multigrid.py covers the boxes geometrically).

4C solves the structural tangent with Belos CG and a MueLu preconditioner
(4C_solver_nonlin_nox_linearsystem.cpp:275-353, 4C_linear_solver_preconditioner_muelu.cpp); MueLu
(Trilinos sha 06db4c85) is not vendored, so its default smoothed-aggregation setup is restated from
the published algorithm (Vanek, Mandel, Brezina 1996; the steps are in fcg_amg_setup.cpp):

  nodes          the block rows of K (3 DOFs; 6 on the coarse levels = the rigid-body modes)
  aggregation    uncoupled (phases 1 / 2 / 3) on the block graph, drop tolerance 0 (MueLu's
                 default); nodes whose 3 DOFs are all Dirichlet are not aggregated
  near-null sp.  the 6 rigid-body modes of the node coordinates (Dirichlet DOF rows zeroed)
  tentative T    per aggregate QR of the stacked modes: T = Q, coarse near-null space = R
  prolongator    P = (I - omega D^-1 A) T, omega = 4/3 / lambda_max(D^-1 A), D = nodal blocks
  coarse op.     A_c = P^T (A P), recursively until <= coarse_max DOFs; the coarsest level is
                 factored densely (Cholesky inverse on the device, applied as one GEMV)
  cycle          the V-cycle and flexible CG of multigrid.CycleFCG: Chebyshev(nu) in D^-1 A on
                 every level but the coarsest, lambda_max from the Lanczos estimate

Graph work (aggregation, QR of the near-null space, the symbolic products and transposes) is done
once per mesh on the host in C++ (the patterns do not change between tangents); every numeric step
-- the BSR copy of K, the block inverses, the three products per level, the smoothing, the dense
coarsest factor -- is recomputed on the device for each tangent by the library's fcg_bsr_* /
fcg_amg_* kernels (fcg_amg.hip).  torch supplies the buffers, the vector updates and the small
dense Cholesky of the coarsest level."""

import ctypes
import time

import numpy as np
import torch

from . import fcg
from .multigrid import CycleFCG, _Level, _LevelOps

_NM = 6  # near-null-space modes (3D elasticity: 3 translations + 3 rotations)


def _vp(a):
    """ctypes pointer of a numpy array or torch tensor (None -> NULL)."""
    if a is None:
        return None
    if isinstance(a, torch.Tensor):
        return ctypes.c_void_p(a.data_ptr())
    return ctypes.c_void_p(a.ctypes.data)


def _check(rc, what):
    if rc != 0:
        raise fcg.FcgError(rc, what)


# -- host graph steps (C++ in the library; numpy arrays in and out) ---------------------------
def aggregate(ptr, col, skip=None):
    """Uncoupled aggregation of the block graph (ptr, col): (agg int32 [-1 = not aggregated], n_agg)."""
    ptr = np.ascontiguousarray(ptr, dtype=np.int64)
    col = np.ascontiguousarray(col, dtype=np.int32)
    n = len(ptr) - 1
    sk = None if skip is None else np.ascontiguousarray(skip, dtype=np.uint8)
    agg = np.empty(n, dtype=np.int32)
    n_agg = fcg.lib().fcg_amg_aggregate(n, _vp(ptr), _vp(col), _vp(sk), _vp(agg))
    if n_agg < 0:
        raise ValueError("fcg_amg_aggregate: bad graph")
    return agg, int(n_agg)


def tentative(ns, agg, n_agg):
    """Tentative prolongator blocks [n][bs][6] and coarse near-null space [n_agg][6][6] from the
    near-null space ns [n][bs][6]; also the count of vanished (rank-deficient) columns."""
    ns = np.ascontiguousarray(ns, dtype=np.float64)
    n, bs = ns.shape[0], ns.shape[1]
    agg = np.ascontiguousarray(agg, dtype=np.int32)
    tv = np.empty((n, bs, _NM))
    nsc = np.empty((n_agg, _NM, _NM))
    nd = ctypes.c_int64(0)
    _check(fcg.lib().fcg_amg_tentative(n, bs, _vp(ns), _vp(agg), n_agg, _vp(tv), _vp(nsc),
                                       ctypes.byref(nd)), "fcg_amg_tentative")
    return tv, nsc, int(nd.value)


def symbolic(a_ptr, a_col, b_ptr, b_col, n_cols):
    """Block pattern (ptr, col) of A B."""
    L = fcg.lib()
    a_ptr, b_ptr = (np.ascontiguousarray(p, dtype=np.int64) for p in (a_ptr, b_ptr))
    a_col, b_col = (np.ascontiguousarray(c, dtype=np.int32) for c in (a_col, b_col))
    n = len(a_ptr) - 1
    c_ptr = np.empty(n + 1, dtype=np.int64)
    nnz = L.fcg_bsr_symbolic(n, _vp(a_ptr), _vp(a_col), _vp(b_ptr), _vp(b_col), n_cols,
                             _vp(c_ptr), None)
    if nnz < 0:
        raise ValueError("fcg_bsr_symbolic: bad pattern")
    c_col = np.empty(max(nnz, 1), dtype=np.int32)
    if L.fcg_bsr_symbolic(n, _vp(a_ptr), _vp(a_col), _vp(b_ptr), _vp(b_col), n_cols, _vp(c_ptr),
                          _vp(c_col)) != nnz:
        raise ValueError("fcg_bsr_symbolic: fill pass disagrees with the count pass")
    return c_ptr, c_col[:nnz]


def product_plan(a_ptr, a_col, b_ptr, b_col, c_ptr, c_col, n_cols):
    """fcg_bsr_product_plan: per block of C = A B on C's pattern its (A block, B block) pairs in
    A's row order -> (pair_ptr, pair_a, pair_b)."""
    L = fcg.lib()
    a_ptr, b_ptr, c_ptr = (np.ascontiguousarray(p, dtype=np.int64) for p in (a_ptr, b_ptr, c_ptr))
    a_col, b_col, c_col = (np.ascontiguousarray(c, dtype=np.int32) for c in (a_col, b_col, c_col))
    n = len(a_ptr) - 1
    pp = np.empty(int(c_ptr[-1]) + 1, dtype=np.int64)
    npairs = L.fcg_bsr_product_plan(n, _vp(a_ptr), _vp(a_col), _vp(b_ptr), _vp(b_col), _vp(c_ptr),
                                    _vp(c_col), n_cols, _vp(pp), None, None)
    if npairs < 0:
        raise ValueError("fcg_bsr_product_plan: bad pattern")
    pa, pb = np.empty(max(npairs, 1), dtype=np.int32), np.empty(max(npairs, 1), dtype=np.int32)
    if L.fcg_bsr_product_plan(n, _vp(a_ptr), _vp(a_col), _vp(b_ptr), _vp(b_col), _vp(c_ptr),
                              _vp(c_col), n_cols, _vp(pp), _vp(pa), _vp(pb)) != npairs:
        raise ValueError("fcg_bsr_product_plan: fill pass disagrees with the count pass")
    return pp, pa[:npairs], pb[:npairs]


def transpose_pattern(ptr, col, n_cols):
    """Pattern of A^T and perm (transposed block -> A's block index)."""
    ptr = np.ascontiguousarray(ptr, dtype=np.int64)
    col = np.ascontiguousarray(col, dtype=np.int32)
    nnz = int(ptr[-1])
    t_ptr = np.empty(n_cols + 1, dtype=np.int64)
    t_col = np.empty(max(nnz, 1), dtype=np.int32)
    perm = np.empty(max(nnz, 1), dtype=np.int64)
    _check(fcg.lib().fcg_bsr_transpose_pattern(len(ptr) - 1, n_cols, _vp(ptr), _vp(col), _vp(t_ptr),
                                               _vp(t_col), _vp(perm)), "fcg_bsr_transpose_pattern")
    return t_ptr, t_col[:nnz], perm[:nnz]


def rigid_body_modes(x):
    """[n][3][6] near-null space of 3D elasticity at the points x [n][3] (about their centroid):
    translations x, y, z, then rotations about z, x, y."""
    x = np.asarray(x, dtype=np.float64)
    c = x - x.mean(axis=0)
    n = len(x)
    B = np.zeros((n, 3, _NM))
    B[:, 0, 0] = B[:, 1, 1] = B[:, 2, 2] = 1.0
    B[:, 0, 3], B[:, 1, 3] = -c[:, 1], c[:, 0]
    B[:, 1, 4], B[:, 2, 4] = -c[:, 2], c[:, 1]
    B[:, 0, 5], B[:, 2, 5] = c[:, 2], -c[:, 0]
    return B


def diag_index(ptr, col):
    """Block index of every row's diagonal block (raises if one is missing)."""
    n = len(ptr) - 1
    rows = np.repeat(np.arange(n, dtype=np.int64), np.diff(ptr))
    hit = np.nonzero(col == rows)[0]
    d = np.full(n, -1, dtype=np.int64)
    d[rows[hit]] = hit
    if (d < 0).any():
        raise ValueError("block row without a diagonal block")
    return d


class Bsr:
    """Block CSR matrix: host pattern (ptr, col), device pattern and values (row-major blocks)."""

    def __init__(self, ptr, col, br, bc, n_cols, dev):
        self.ptr_h = np.ascontiguousarray(ptr, dtype=np.int64)
        self.col_h = np.ascontiguousarray(col, dtype=np.int32)
        self.n, self.nnzb = len(self.ptr_h) - 1, int(self.ptr_h[-1])
        self.br, self.bc, self.n_cols, self.dev = br, bc, n_cols, dev
        self.ptr = torch.from_numpy(self.ptr_h).to(dev)
        self.col = torch.from_numpy(self.col_h).to(dev)
        self.vals = torch.zeros(max(self.nnzb, 1) * br * bc, dtype=torch.float64, device=dev)

    def stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.dev).cuda_stream)

    def spmv(self, x, y, alpha=1.0, accumulate=False):
        _check(fcg.lib().fcg_bsr_spmv(self.dev.index or 0, self.br, self.bc, self.n, _vp(self.ptr),
                                      _vp(self.col), _vp(self.vals), _vp(x), _vp(y), alpha,
                                      1 if accumulate else 0, self.stream()), "fcg_bsr_spmv")

    def product(self, A, B):
        """self = A B (self holds the pattern of the product)."""
        _check(fcg.lib().fcg_bsr_spgemm(self.dev.index or 0, A.br, A.bc, B.bc, A.n, _vp(A.ptr),
                                        _vp(A.col), _vp(A.vals), _vp(B.ptr), _vp(B.col),
                                        _vp(B.vals), _vp(self.ptr), _vp(self.col), _vp(self.vals),
                                        self.stream()), "fcg_bsr_spgemm")

    def to_numpy(self):
        """Dense host copy (tests)."""
        v = self.vals.cpu().numpy()[:self.nnzb * self.br * self.bc].reshape(-1, self.br, self.bc)
        D = np.zeros((self.n * self.br, self.n_cols * self.bc))
        for i in range(self.n):
            for k in range(self.ptr_h[i], self.ptr_h[i + 1]):
                j = self.col_h[k]
                D[i * self.br:(i + 1) * self.br, j * self.bc:(j + 1) * self.bc] = v[k]
        return D


class _BsrLevel(_LevelOps):
    """A coarse level: operator A (6 x 6 blocks), its block-diagonal inverse, work vectors."""

    def __init__(self, A, dev):
        self.A, self.dev = A, dev
        self.n = A.n * A.br
        f64 = dict(dtype=torch.float64, device=dev)
        self.mask = torch.ones(self.n, **f64)
        self.x, self.b, self.r, self.d, self.z = (torch.zeros(self.n, **f64) for _ in range(5))
        self.diag = torch.from_numpy(diag_index(A.ptr_h, A.col_h)).to(dev)
        self.dinv = torch.empty(A.n * A.br * A.br, **f64)
        self.flag = torch.zeros(1, dtype=torch.int32, device=dev)
        self.lmax = None

    def setup_diag(self):
        A = self.A
        rc = fcg.lib().fcg_bsr_block_jacobi_setup(self.dev.index or 0, A.br, A.n, _vp(A.ptr),
                                                  _vp(self.diag), _vp(A.vals), _vp(self.dinv),
                                                  _vp(self.flag), A.stream())
        _check(rc, f"AMG level with {A.n} block rows: singular diagonal block")

    def apply_dinv(self, r, z, scale=1.0, accumulate=False):
        A = self.A
        _check(fcg.lib().fcg_bsr_block_jacobi_apply(self.dev.index or 0, A.br, A.n, _vp(self.dinv),
                                                    _vp(r), _vp(z), scale, 1 if accumulate else 0,
                                                    A.stream()), "fcg_bsr_block_jacobi_apply")

    def spmv(self, x, y):
        self.A.spmv(x, y)

    spmv_exact = spmv


class _DenseLevel(_BsrLevel):
    """The coarsest level: A as a dense matrix, solved by its Cholesky inverse (one GEMV)."""

    def factor(self):
        self.setup_diag()  # unit diagonal on empty rows (vanished near-null-space columns)
        A = self.A
        D = torch.zeros((self.n, self.n), dtype=torch.float64, device=self.dev)
        _check(fcg.lib().fcg_bsr_to_dense(self.dev.index or 0, A.br, A.n, _vp(A.ptr), _vp(A.col),
                                          _vp(A.vals), _vp(D), A.stream()), "fcg_bsr_to_dense")
        D = 0.5 * (D + D.T)
        Lc, info = torch.linalg.cholesky_ex(D)
        if int(info) != 0:
            raise fcg.FcgError(fcg.FCG_ERR_SINGULAR, f"AMG coarsest level ({self.n} DOFs) is not "
                               f"positive definite (Cholesky pivot {int(info)})")
        self.Ainv = torch.cholesky_inverse(Lc)


class _Step:
    """Transfer between level l (block size bs) and l + 1: aggregates, T, P, A T, A P, P^T."""

    def __init__(self, A, agg, n_agg, tent, bs, dev):
        self.bs, self.n_agg = bs, n_agg
        has = agg >= 0
        tptr = np.concatenate([[0], np.cumsum(has)]).astype(np.int64)
        self.T = Bsr(tptr, agg[has], bs, _NM, n_agg, dev)
        self.T.vals[:int(has.sum()) * bs * _NM] = torch.from_numpy(
            np.ascontiguousarray(tent[has]).ravel()).to(dev)
        self.agg = torch.from_numpy(np.ascontiguousarray(agg, dtype=np.int32)).to(dev)
        self.tent = torch.from_numpy(np.ascontiguousarray(tent).ravel()).to(dev)  # every row's T_i
        pp, pc = symbolic(A.ptr_h, A.col_h, tptr, agg[has], n_agg)
        self.P = Bsr(pp, pc, bs, _NM, n_agg, dev)
        self.AT = Bsr(pp, pc, bs, _NM, n_agg, dev)  # A T on P's pattern
        app, apc = symbolic(A.ptr_h, A.col_h, pp, pc, n_agg)
        self.AP = Bsr(app, apc, bs, _NM, n_agg, dev)
        tp, tc, perm = transpose_pattern(pp, pc, n_agg)
        self.Pt = Bsr(tp, tc, _NM, bs, A.n, dev)
        self.perm = torch.from_numpy(perm).to(dev)
        cp, cc = symbolic(tp, tc, app, apc, n_agg)
        self.Ac_pattern = (cp, cc)


class AMG(CycleFCG):
    """Flexible CG preconditioned by a smoothed-aggregation V-cycle (see module doc).

    mesh / ev: the single-rank discretization being solved (fcg.Discretization or BoxMesh and its
    Evaluator); dbc_rows: the Newton's Dirichlet rows (unit rows of K)."""

    # _setup estimates lambda_max afresh for every tangent (same seed) and the prolongators
    # depend on it: a retry would repeat the failed solve exactly, so fail at once
    retry_lmax = False

    def __init__(self, mesh, ev, dbc_rows, nu=2, max_levels=10, coarse_max=3000, omega=4.0 / 3.0,
                 ratio=20.0, boost=1.1):
        info = ev.info
        n_rows = int(info.n_rows)
        if int(info.n_cols) != n_rows or n_rows % 3:
            raise ValueError("AMG is single-rank: the column map must be the row map, 3 DOFs a node")
        nn = n_rows // 3
        ndr = np.asarray(mesh.node_dof_row, dtype=np.int64)
        order = np.argsort(ndr, kind="stable")
        if len(ndr) != nn or not np.array_equal(ndr[order], 3 * np.arange(nn)):
            raise ValueError("AMG needs node-major DOFs: row 3b + d = DOF d of the b-th node")
        dev = torch.device("cuda", ev.device)
        self.dev, self.ev, self.nu, self.ratio, self.boost = dev, ev, nu, ratio, boost
        self.omega, self.trace = omega, False
        self.setup_ms = []  # numeric setup time of every tangent (synchronised wall clock)
        self.rows = np.sort(np.asarray(dbc_rows, dtype=np.int32))
        # level 0 as a block graph: block row b = rows 3b..3b+2 (one pattern of DOF triples)
        rp = np.asarray(mesh.rowptr, dtype=np.int64)
        cl = np.asarray(mesh.col_lid, dtype=np.int32)
        r0 = rp[0:3 * nn:3]
        nb = (rp[1:3 * nn + 1:3] - r0) // 3
        bptr = np.concatenate([[0], np.cumsum(nb)]).astype(np.int64)
        off = np.arange(int(bptr[-1]), dtype=np.int64) - np.repeat(bptr[:-1], nb)
        bcol = (cl[np.repeat(r0, nb) + 3 * off] // 3).astype(np.int32)
        self.rowptr = torch.from_numpy(rp).to(dev)
        self.A0 = Bsr(bptr, bcol, 3, 3, nn, dev)
        self.A0_diag = torch.from_numpy(diag_index(bptr, bcol)).to(dev)
        self.A0_dinv = torch.empty(9 * nn, dtype=torch.float64, device=dev)
        self.flag = torch.zeros(1, dtype=torch.int32, device=dev)
        dbc = np.zeros(n_rows, dtype=bool)
        dbc[self.rows] = True
        skip = dbc.reshape(nn, 3).all(axis=1)
        ns = rigid_body_modes(np.asarray(mesh.node_x, dtype=np.float64)[order])
        ns[dbc.reshape(nn, 3)] = 0.0
        # symbolic hierarchy
        self.levels = [_Level(mesh, ev, None, self.rows, dev)]
        self.steps = []
        self.deficient = []
        A, bs = self.A0, 3
        # at least one aggregation level, then coarsen until the level is small enough to factor
        while (A.n * bs > coarse_max or not self.steps) and len(self.levels) < max_levels:
            agg, n_agg = aggregate(A.ptr_h, A.col_h, skip)
            if n_agg == 0 or n_agg >= A.n:
                break
            tent, ns, nd = tentative(ns, agg, n_agg)
            st = _Step(A, agg, n_agg, tent, bs, dev)
            self.steps.append(st)
            self.deficient.append(nd)
            A = Bsr(st.Ac_pattern[0], st.Ac_pattern[1], _NM, _NM, n_agg, dev)
            self.levels.append(_BsrLevel(A, dev))
            bs, skip = _NM, None
        if len(self.levels) < 2:
            raise ValueError(f"AMG: no coarse level for {n_rows} DOFs (coarse_max {coarse_max})")
        last = self.levels[-1]
        self.levels[-1] = _DenseLevel(last.A, dev)
        if self.levels[-1].n > 20000:
            raise ValueError(f"AMG: coarsest level has {self.levels[-1].n} DOFs (raise max_levels)")

    def describe(self):
        out = [{"level": 0, "dofs": self.levels[0].n, "block_rows": self.A0.n,
                "blocks": self.A0.nnzb, "lmax": self.levels[0].lmax}]
        for l, st in enumerate(self.steps, start=1):
            lv = self.levels[l]
            out.append({"level": l, "dofs": lv.n, "block_rows": lv.A.n, "blocks": lv.A.nnzb,
                        "P_blocks": st.P.nnzb, "deficient": self.deficient[l - 1],
                        "lmax": lv.lmax, "dense": isinstance(lv, _DenseLevel)})
        return out

    def check_dirichlet(self, dbc_rows):
        theirs = np.sort(np.asarray(dbc_rows, dtype=np.int32))
        if not np.array_equal(self.rows, theirs):
            raise ValueError(f"AMG Dirichlet rows ({len(self.rows)}) differ from the system's "
                             f"({len(theirs)})")

    # -- numeric setup for a tangent ----------------------------------------------------------
    def _prepare(self, K):
        torch.cuda.synchronize(self.dev)
        t0 = time.perf_counter()
        self._setup(K)
        torch.cuda.synchronize(self.dev)
        self.setup_ms.append(1e3 * (time.perf_counter() - t0))

    def _setup(self, K):
        L, dev = fcg.lib(), self.dev.index or 0
        f0 = self.levels[0]
        f0.K = K
        f0.setup_diag()
        f0.estimate_lmax()
        s = self.A0.stream()
        _check(L.fcg_bsr_from_node_csr(dev, self.A0.n, _vp(self.rowptr), _vp(self.A0.ptr), _vp(K),
                                       _vp(self.A0.vals), s), "fcg_bsr_from_node_csr")
        _check(L.fcg_bsr_block_jacobi_setup(dev, 3, self.A0.n, _vp(self.A0.ptr), _vp(self.A0_diag),
                                            _vp(self.A0.vals), _vp(self.A0_dinv), _vp(self.flag), s),
               "singular nodal diagonal block of K")
        A, dinv = self.A0, self.A0_dinv
        for l, st in enumerate(self.steps):
            lv = self.levels[l]
            st.AT.product(A, st.T)
            _check(L.fcg_amg_smooth_prolongator(dev, st.bs, A.n, _vp(st.P.ptr), _vp(st.P.col),
                                                _vp(st.agg), _vp(st.tent), _vp(dinv),
                                                _vp(st.AT.vals), self.omega / lv.lmax,
                                                _vp(st.P.vals), s), "fcg_amg_smooth_prolongator")
            st.AP.product(A, st.P)
            _check(L.fcg_bsr_transpose_values(dev, st.bs, _NM, st.P.nnzb, _vp(st.perm),
                                              _vp(st.P.vals), _vp(st.Pt.vals), s),
                   "fcg_bsr_transpose_values")
            c = self.levels[l + 1]
            c.A.product(st.Pt, st.AP)
            if isinstance(c, _DenseLevel):
                c.factor()
            else:
                c.setup_diag()
                c.estimate_lmax()
            A, dinv = c.A, c.dinv

    def _restrict(self, l, r, cb):
        self.steps[l].Pt.spmv(r, cb)

    def _prolong(self, l, cx, x):
        self.steps[l].P.spmv(cx, x, accumulate=True)

    def _coarse_solve(self, lvl, b, x):
        torch.mv(lvl.Ainv, b, out=x)


class NativeAMG:
    """The same smoothed-aggregation AMG solve as one native object behind the C ABI
    (fcg_amg_create / fcg_amg_solve, fcg_amg_solver.hip) -- what a C++ host calls; the coarsest
    level is solved by block-Jacobi CG to coarse_rtol instead of a dense factor.  Same interface
    as AMG: solve(K, b, x, rtol, max_iter) -> (iterations, relative residual)."""

    def __init__(self, mesh, ev, dbc_rows, **opts):
        """On a rank of a multi-rank partition (column map = owned DOFs first, then ghosts) the
        AMG is built on the rank's owned block: the local preconditioner of dsolve.NativeDFCG."""
        L = fcg.lib()
        info = ev.info
        n_rows = int(info.n_rows)
        if n_rows % 3:
            raise ValueError("NativeAMG needs 3 DOFs per owned node")
        ndr_all = np.asarray(mesh.node_dof_row, dtype=np.int64)
        own = np.nonzero(ndr_all >= 0)[0]
        ndr = ndr_all[own]
        order = own[np.argsort(ndr, kind="stable")]
        if not np.array_equal(ndr_all[order], 3 * np.arange(n_rows // 3)):
            raise ValueError("NativeAMG needs node-major DOFs: row 3b + d = DOF d of the b-th node")
        self.ev, self.dev = ev, torch.device("cuda", ev.device)
        self.rows = np.sort(np.asarray(dbc_rows, dtype=np.int32))
        self._rowptr = np.ascontiguousarray(mesh.rowptr, dtype=np.int64)
        self._col = np.ascontiguousarray(mesh.col_lid, dtype=np.int32)
        self._x = np.ascontiguousarray(np.asarray(mesh.node_x, dtype=np.float64)[order])
        self.opt = fcg.FcgAmgOptions()
        L.fcg_amg_default_options(ctypes.byref(self.opt))
        for k, v in opts.items():
            setattr(self.opt, k, v)
        h = ctypes.c_void_p()
        rc = L.fcg_amg_create(ev._h, _vp(self._rowptr), _vp(self._col), _vp(self._x), len(self.rows),
                              _vp(self.rows), ctypes.byref(self.opt), ctypes.byref(h))
        if rc != 0:
            raise fcg.FcgError(rc, L.fcg_last_error(ev._h).decode())
        self._h = h
        self.setup_ms = []
        # a rank of a partition: the handle preconditions the solve across ranks only
        self.local = int(info.n_cols) != n_rows

    def close(self):
        if getattr(self, "_h", None):
            fcg.lib().fcg_amg_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def check_dirichlet(self, dbc_rows):
        theirs = np.sort(np.asarray(dbc_rows, dtype=np.int32))
        if not np.array_equal(self.rows, theirs):
            raise ValueError("NativeAMG Dirichlet rows differ from the system's")

    def describe(self):
        L = fcg.lib()
        out = []
        for l in range(L.fcg_amg_levels(self._h)):
            d, b, lm = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_double()
            L.fcg_amg_level_info(self._h, l, ctypes.byref(d), ctypes.byref(b), ctypes.byref(lm))
            out.append({"level": l, "dofs": d.value, "blocks": b.value, "lmax": lm.value})
        return out

    def stats(self):
        """fcg_amg_stats: whether the coarsest level is a dense inverse, graph-replayed iterations."""
        dense, launches = ctypes.c_int(0), ctypes.c_int(0)
        fcg.lib().fcg_amg_stats(self._h, ctypes.byref(dense), ctypes.byref(launches))
        return {"coarse_dense": bool(dense.value), "graph_launches": launches.value}

    def setup(self, K):
        """Numeric setup for the tangent K (fcg_amg_setup)."""
        L = fcg.lib()
        s = ctypes.c_void_p(torch.cuda.current_stream(self.dev).cuda_stream)
        rc = L.fcg_amg_setup(self._h, _vp(K), s)
        if rc != 0:
            raise fcg.FcgError(rc, L.fcg_amg_last_error(self._h).decode())
        self.setup_ms.append(L.fcg_amg_setup_ms(self._h))

    def solve(self, K, b, x, rtol, max_iter=1000, setup=True):
        """K x = b from x = 0; setup=False iterates on the last setup (a constant operator)."""
        L = fcg.lib()
        if self.local:
            # the library refuses it too (fcg_amg_iterate: FCG_ERR_ARG); say so before any setup
            raise fcg.FcgError(3, "NativeAMG.solve: multi-rank context -- solve across ranks with "
                               "dsolve.NativeDFCG (fcg_dfcg_solve); this AMG is its preconditioner")
        if setup:
            self.setup(K)
        it, rel = ctypes.c_int(0), ctypes.c_double(0.0)
        s = ctypes.c_void_p(torch.cuda.current_stream(self.dev).cuda_stream)
        rc = L.fcg_amg_iterate(self._h, _vp(K), _vp(b), _vp(x), float(rtol), int(max_iter),
                               ctypes.byref(it), ctypes.byref(rel), s)
        if rc != 0:
            raise fcg.FcgError(rc, L.fcg_amg_last_error(self._h).decode())
        return it.value, rel.value
