"""Geometric multigrid preconditioner for the Newton solve on GridGenerator boxes (SURVEY §8f
row 2: "GPU CG with a Jacobi/AMG preconditioner").

4C hands the linearised system to Belos with a MueLu (smoothed-aggregation AMG) preconditioner
(4C_solver_nonlin_nox_linearsystem.cpp:275-353, 4C_linear_solver_preconditioner_muelu.cpp).
MueLu is not vendored and builds its hierarchy from the matrix graph; on the structured boxes of
the BASELINE configs the hierarchy is known in advance, so it is built geometrically instead:

  level 0   the tangent K being solved (hex27 or hex8, any kinematics, Dirichlet unit rows)
  level 1   hex27 -> hex8 on the same elements (p-coarsening), if level 0 is hex27
  level l+1 hex8 n -> hex8 (n+1)/2 (h-coarsening) while that stays >= min_intervals (an odd n
            gives a non-nested level: trilinear interpolation at general weights)

Coarse operators are rediscretised: linear-elastic StVK hex8 assembled by the library's own
evaluate (for affine boxes and linear kinematics this is exactly the Galerkin product P^T K P,
the quadrature being exact for the trilinear subspace).  Transfers are the nodal interpolation of
a trilinear field (weights 1 or 1/2 per direction) and its transpose, applied by
fcg_node_transfer.  Smoother: Chebyshev polynomial in D^-1 K with D the 3x3 nodal diagonal blocks
(Ifpack2's Chebyshev with point-block diagonal, boost 1.1 as Ifpack2's; eigenvalue ratio 10 instead of
Ifpack2's 30: 54 FCG iterations for config 3's four Newton steps against 60 at 20 and 71 at 30),
the same polynomial before and after the coarse correction.  Coarsest level: block-Jacobi PCG to a
loose tolerance -- a nonlinear preconditioner, so the outer iteration is flexible CG
(Polak-Ribiere beta).  Every level's K, the work vectors and the transfer tables stay in HBM;
torch supplies the buffers and the vector updates (axpy, dot), the library the operator, the
smoother's block-diagonal solve and the transfers.  With mixed=True the fine level's Chebyshev
smoother SpMVs (3 of the 5 per iteration) read an FP32 copy of K (fcg_spmv_f32); the outer
flexible CG's SpMV and the residual restricted to the coarse level stay FP64.  Off by default:
on the hex27 TotLag cantilever of tests/test_multigrid.py it raised the FCG iterations to a
1e-12 tolerance from below 525 to 888.
"""

import ctypes
import os
import sys
import time

import numpy as np
import torch

from . import fcg


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr())


def node_lattice(mesh):
    """(i, j, k) of every node on the mesh's own node lattice (GridGenerator node GIDs,
    4C_io_gridgenerator.cpp:283-291: gid = (ez NY + ey) NX + ex on the 2n+1 lattice; hex8 nodes
    sit at its even points)."""
    iv = [int(mesh.box.interval[d]) for d in range(3)]
    NX, NY = 2 * iv[0] + 1, 2 * iv[1] + 1
    g = mesh.node_gid - int(mesh.box.first_node_gid)
    ijk = np.stack([g % NX, (g // NX) % NY, g // (NX * NY)], axis=1)
    if mesh.celltype == fcg.HEX8:
        ijk //= 2
    return ijk


def transfer_tables(fine, coarse):
    """Prolongation fine <- coarse (trilinear nodal interpolation) and its transpose, as
    node-block tables for fcg_node_transfer: (ptr, src_row0, w, dst_row0) each.  Both meshes
    span the same GridGenerator box; a fine node at lattice index f of N_f points sits at coarse
    lattice coordinate f (N_c - 1) / (N_f - 1) -- on a 2:1 refinement the weights are 1 or 1/2,
    otherwise (an odd interval count halved to (n + 1) / 2) the general linear weights."""
    fl, cl = node_lattice(fine), node_lattice(coarse)
    cdim = cl.max(axis=0) + 1
    fdim = fl.max(axis=0) + 1
    if (cdim > fdim).any() or (cdim < 2).any():
        raise ValueError("coarse lattice is not coarser than the fine one")
    crow = np.full(tuple(cdim), -1, dtype=np.int64)
    crow[cl[:, 0], cl[:, 1], cl[:, 2]] = coarse.node_dof_row
    nf = len(fl)
    lo, hi, wl, wh = [], [], [], []
    for d in range(3):
        c = fl[:, d] * float(cdim[d] - 1) / float(fdim[d] - 1)
        i0 = np.minimum(np.floor(c).astype(np.int64), cdim[d] - 2)
        t = c - i0
        lo.append(i0)
        hi.append(i0 + 1)
        wl.append(1.0 - t)
        wh.append(t)
    fidx, cidx, w = [], [], []
    for cx in range(2):
        for cy in range(2):
            for cz in range(2):
                wx = wh[0] if cx else wl[0]
                wy = wh[1] if cy else wl[1]
                wz = wh[2] if cz else wl[2]
                ww = wx * wy * wz
                m = ww > 0
                ix = (hi[0] if cx else lo[0])[m]
                iy = (hi[1] if cy else lo[1])[m]
                iz = (hi[2] if cz else lo[2])[m]
                fidx.append(np.nonzero(m)[0])
                cidx.append(crow[ix, iy, iz])
                w.append(ww[m])
    fidx, cidx, w = np.concatenate(fidx), np.concatenate(cidx), np.concatenate(w)
    if (cidx < 0).any():
        raise ValueError("coarse node missing from the coarse mesh")
    frow = fine.node_dof_row.astype(np.int64)

    def table(out_idx, out_row, src_row, n_out):
        order = np.lexsort((src_row, out_idx))
        ptr = np.zeros(n_out + 1, dtype=np.int64)
        np.add.at(ptr, out_idx + 1, 1)
        return (np.cumsum(ptr), src_row[order].astype(np.int32), w[order].copy(),
                out_row.astype(np.int32))

    # prolongation: out = fine nodes, sources = coarse rows
    P = table(fidx, frow, cidx, nf)
    # restriction (transpose): out = coarse nodes (numbered by the coarse mesh's node index)
    cl_of_entry = np.empty(len(cidx), dtype=np.int64)
    # coarse node index of every entry: invert crow (row0 -> node) through a dense map
    row2node = np.full(int(coarse.node_dof_row.max()) + 1, -1, dtype=np.int64)
    row2node[coarse.node_dof_row] = np.arange(len(cl))
    cl_of_entry[:] = row2node[cidx]
    R = table(cl_of_entry, coarse.node_dof_row.astype(np.int64), frow[fidx], len(cl))
    return P, R


def box_stencil(mesh, youngs, poisson, device, dbc_rows):
    """The 27-point stencil of a rediscretised hex8 GridGenerator box (all elements the same
    parallelepiped, linear StVK) for fcg_box_stencil_apply: (nx, ny, nz, row_of, clamped, S) with
    S[27 node classes][27 offsets][3 x 3] summed from the element matrix, which the library
    assembles on a one-element box of the same size and rotation."""
    box = mesh.box
    iv = [int(box.interval[d]) for d in range(3)]
    if min(iv) < 1:
        raise ValueError("box stencil: empty box")
    h = [(box.upper[d] - box.lower[d]) / iv[d] for d in range(3)]
    one = fcg.BoxMesh(fcg.HEX8, (1, 1, 1), lower=(0.0, 0.0, 0.0), upper=tuple(h),
                      rotation=tuple(box.rotation[d] for d in range(3)))
    ev = fcg.Evaluator(one, kinematics=fcg.LINEAR, youngs=youngs, poisson=poisson, device=device.index or 0)
    f64 = dict(dtype=torch.float64, device=device)
    K = torch.zeros(one.nnz, **f64)
    ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, torch.zeros(one.n_cols, **f64),
                       torch.zeros(one.n_rows, **f64), K)
    Kh = K.cpu().numpy()
    ev.close()
    A = np.zeros((one.n_rows, one.n_cols))
    A[np.repeat(np.arange(one.n_rows), np.diff(one.rowptr)), one.col_lid] = Kh
    lat1 = node_lattice(one)
    row1 = {tuple(int(v) for v in lat1[n]): int(one.node_dof_row[n]) for n in range(len(lat1))}
    S = np.zeros((27, 27, 3, 3))
    for cls in range(27):
        c = (cls % 3, (cls // 3) % 3, cls // 9)
        for ea in range(2):
            for eb in range(2):
                for ec in range(2):
                    e = (ea, eb, ec)
                    if any((c[d] == 0 and e[d] == 0) or (c[d] == 2 and e[d] == 1) for d in range(3)):
                        continue
                    rn = row1[(1 - ea, 1 - eb, 1 - ec)]
                    for p in range(2):
                        for q in range(2):
                            for r in range(2):
                                o = (ea - 1 + p) + 1 + 3 * ((eb - 1 + q) + 1) + 9 * ((ec - 1 + r) + 1)
                                rm = row1[(p, q, r)]
                                S[cls, o] += A[rn:rn + 3, rm:rm + 3]
    lat = node_lattice(mesh)
    nx, ny, nz = iv[0] + 1, iv[1] + 1, iv[2] + 1
    row_of = np.full(nx * ny * nz, -1, dtype=np.int32)
    idx = lat[:, 0] + nx * (lat[:, 1] + ny * lat[:, 2])
    row_of[idx] = mesh.node_dof_row
    clamped = np.zeros(nx * ny * nz, dtype=np.uint8)
    dbc = np.asarray(dbc_rows, dtype=np.int64)
    if len(dbc):
        is_dbc = np.zeros(mesh.n_rows, dtype=bool)
        is_dbc[dbc] = True
        ok = mesh.node_dof_row >= 0
        full = np.zeros(len(lat), dtype=bool)
        r0 = mesh.node_dof_row[ok]
        full[ok] = is_dbc[r0] & is_dbc[r0 + 1] & is_dbc[r0 + 2]
        part = np.zeros(len(lat), dtype=bool)
        part[ok] = (is_dbc[r0] | is_dbc[r0 + 1] | is_dbc[r0 + 2]) & ~full[ok]
        if part.any():
            return None  # a node with some of its DOFs clamped: no unit-row node class for it
        clamped[idx[full]] = 1
    return (nx, ny, nz, torch.from_numpy(row_of).to(device), torch.from_numpy(clamped).to(device),
            torch.from_numpy(S.ravel()).to(device))


class _Transfer:
    def __init__(self, tab, device):
        ptr, src, w, dst = tab
        self.n_out = len(dst)
        self.ptr = torch.from_numpy(ptr).to(device)
        self.src = torch.from_numpy(src).to(device)
        self.w = torch.from_numpy(w).to(device)
        self.dst = torch.from_numpy(dst).to(device)
        self.device = device.index or 0

    def __call__(self, x, y, accumulate):
        rc = fcg.lib().fcg_node_transfer(
            self.device, ctypes.c_int64(self.n_out), _ptr(self.ptr), _ptr(self.src), _ptr(self.w),
            _ptr(self.dst), _ptr(x), _ptr(y), 1 if accumulate else 0,
            ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream))
        if rc != 0:
            raise fcg.FcgError(rc, "fcg_node_transfer failed")


def _lattice_rows(mesh, rows):
    """(dims, row_of[lattice], node_dirichlet[lattice]) of a box mesh: the row LID of each lattice
    point's first DOF and whether all its DOFs are Dirichlet rows (None when some node is only
    partly constrained)."""
    lat = node_lattice(mesh)
    dims = lat.max(axis=0) + 1
    idx = lat[:, 0] + dims[0] * (lat[:, 1] + dims[1] * lat[:, 2])
    row_of = np.full(int(np.prod(dims)), -1, dtype=np.int32)
    row_of[idx] = mesh.node_dof_row
    is_dbc = np.zeros(mesh.n_rows, dtype=bool)
    is_dbc[np.asarray(rows, dtype=np.int64)] = True
    ok = mesh.node_dof_row >= 0
    r0 = mesh.node_dof_row[ok]
    cnt = is_dbc[r0].astype(int) + is_dbc[r0 + 1] + is_dbc[r0 + 2]
    if ((cnt > 0) & (cnt < 3)).any():
        return None
    zero = np.zeros(len(row_of), dtype=np.uint8)
    zero[idx[ok][cnt == 3]] = 1
    return dims, row_of, zero


class _BoxTransfer:
    """fcg_box_transfer between a box level and its 2:1 coarsening, the level masks applied in the
    kernel (prolong: the fine level's Dirichlet rows, restrict: the coarse level's)."""

    def __init__(self, fine, frows, coarse, crows, device):
        f, c = _lattice_rows(fine, frows), _lattice_rows(coarse, crows)
        if f is None or c is None or not np.array_equal(f[0], 2 * c[0] - 1) or (c[0] < 2).any():
            raise ValueError("not a 2:1 box pair with node-wise Dirichlet rows")
        self.fd, self.cd = [int(v) for v in f[0]], [int(v) for v in c[0]]
        self.frow, self.fzero = (torch.from_numpy(a).to(device) for a in f[1:])
        self.crow, self.czero = (torch.from_numpy(a).to(device) for a in c[1:])
        self.device = device.index or 0

    def _run(self, mode, zero, x, y, accumulate):
        rc = fcg.lib().fcg_box_transfer(self.device, mode, *self.fd, *self.cd, _ptr(self.frow),
                                        _ptr(self.crow), _ptr(zero), _ptr(x), _ptr(y),
                                        1 if accumulate else 0,
                                        ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream))
        if rc != 0:
            raise fcg.FcgError(rc, "fcg_box_transfer failed")

    def prolong(self, xc, xf):
        self._run(0, self.fzero, xc, xf, True)

    def restrict(self, rf, bc):
        self._run(1, self.czero, rf, bc, False)


class _LevelOps:
    """What the Chebyshev smoother and the Lanczos estimate need of a level: n, dev, mask, the
    work vectors r and z, spmv(x, y) and apply_dinv(r, z, scale, accumulate)."""

    def spmv_cycle(self, x, y):
        """The operator of the V-cycle's residual before restriction (FP64)."""
        self.spmv_exact(x, y)

    def estimate_lmax(self, iters=10, seed=20251015):
        """Largest eigenvalue of D^-1 K from the Lanczos tridiagonal of a short block-Jacobi PCG
        run on a random right-hand side (the CG estimate of hypre / AmgX Chebyshev smoothers;
        power iteration converges from below too slowly on these spectra)."""
        # the random start vector is drawn on the device (a host draw of 24M values and its
        # upload took ~0.2 s of config 3's first solve)
        g = torch.Generator(device=self.dev).manual_seed(seed)
        b = (torch.rand(self.n, generator=g, dtype=torch.float64, device=self.dev) - 0.5) * self.mask
        r = b.clone()
        z, q = self.z, self.r
        self.apply_dinv(r, z)
        p = z.clone()
        rz = float(torch.dot(r, z))
        alphas, betas = [], []
        for _ in range(iters):
            self.spmv(p, q)
            pq = float(torch.dot(p, q))
            if not pq > 0.0:
                if not alphas:
                    raise FloatingPointError(
                        f"Lanczos estimate: p.Kp = {pq} on level with {self.n} rows (r.z = {rz}, "
                        f"|p| = {float(torch.linalg.vector_norm(p))}, |Kp| = {float(torch.linalg.vector_norm(q))})")
                break
            alpha = rz / pq
            r.add_(q, alpha=-alpha)
            self.apply_dinv(r, z)
            rz_n = float(torch.dot(r, z))
            alphas.append(alpha)
            if not rz_n > 0.0:
                break
            betas.append(rz_n / rz)
            p.mul_(rz_n / rz).add_(z)
            rz = rz_n
        k = len(alphas)
        T = np.zeros((k, k))
        for i in range(k):
            T[i, i] = 1.0 / alphas[i] + (betas[i - 1] / alphas[i - 1] if i > 0 else 0.0)
            if i + 1 < k:
                T[i, i + 1] = T[i + 1, i] = np.sqrt(betas[i]) / alphas[i]
        self.lmax = float(np.linalg.eigvalsh(T)[-1])


class _Level(_LevelOps):
    def __init__(self, mesh, ev, K, dbc_rows, device):
        self.mesh, self.ev, self.K = mesh, ev, K
        self.rows = np.asarray(dbc_rows, dtype=np.int32)
        self.n = mesh.n_rows
        self.dev = device
        f64 = dict(dtype=torch.float64, device=device)
        self.dinv = torch.empty(9 * (self.n // 3), **f64)
        self.mask = torch.ones(self.n, **f64)
        if len(dbc_rows):
            self.mask[torch.as_tensor(np.asarray(dbc_rows, dtype=np.int64), device=device)] = 0.0
        self.x, self.b, self.r, self.d, self.z = (torch.zeros(self.n, **f64) for _ in range(5))
        self.lmax = None
        self.K32 = None  # FP32 copy of K for the smoother and the V-cycle residual (mixed=True)
        # matrix-free operator (Multigrid(matrix_free=True), hex27 StVK): K(u) x by
        # fcg_tangent_apply at the state set_state gave, the Dirichlet rows as unit rows
        self.matrix_free = False
        self.mf_u = None
        self.stencil = None  # rediscretised box levels: fcg_box_stencil_apply instead of K
        self.mf_dbc = torch.as_tensor(np.asarray(dbc_rows, dtype=np.int64), device=device)

    def stream(self):
        return torch.cuda.current_stream(self.dev)

    def setup_diag(self):
        rc = fcg.lib().fcg_block_jacobi_setup(self.ev._h, _ptr(self.K), _ptr(self.dinv),
                                              ctypes.c_void_p(self.stream().cuda_stream))
        if rc != 0:
            self.ev._raise(rc, -1)

    def apply_dinv(self, r, z, scale=1.0, accumulate=False):
        rc = fcg.lib().fcg_block_jacobi_apply(self.ev._h, _ptr(self.dinv), _ptr(r), _ptr(z),
                                              ctypes.c_double(scale), 1 if accumulate else 0,
                                              ctypes.c_void_p(self.stream().cuda_stream))
        if rc != 0:
            self.ev._raise(rc, -1)

    def cheb_step(self, b, y, d, x, c_d, c_r, mode):
        """One Chebyshev update of d and x from r = b - y (fcg_chebyshev_step; mode 2: from x = 0)."""
        rc = fcg.lib().fcg_chebyshev_step(self.ev._h, _ptr(self.dinv), _ptr(b),
                                          None if y is None else _ptr(y), _ptr(d), _ptr(x),
                                          ctypes.c_double(c_d), ctypes.c_double(c_r), int(mode),
                                          ctypes.c_void_p(self.stream().cuda_stream))
        if rc != 0:
            self.ev._raise(rc, -1)

    def spmv(self, x, y):
        """The V-cycle's operator: K, its FP32 copy when the level has one, (matrix_free) the
        element-by-element tangent action, or (stencil) the box's 27-point stencil."""
        if self.matrix_free:
            self.apply_matrix_free(x, y)
        elif self.stencil is not None:
            self.spmv_exact(x, y)
        elif self.K32 is not None:
            self.ev.spmv_f32(self.K32, x, y, stream=self.stream())
        else:
            self.ev.spmv(self.K, x, y, stream=self.stream())

    def spmv_exact(self, x, y):
        if self.stencil is not None:
            nx, ny, nz, row_of, clamped, S = self.stencil
            rc = fcg.lib().fcg_box_stencil_apply(self.dev.index or 0, nx, ny, nz, _ptr(row_of),
                                                 _ptr(clamped), _ptr(S), _ptr(x), _ptr(y),
                                                 ctypes.c_void_p(self.stream().cuda_stream))
            if rc != 0:
                raise fcg.FcgError(rc, "fcg_box_stencil_apply failed")
            return
        self.ev.spmv(self.K, x, y, stream=self.stream())

    def spmv_cycle(self, x, y):
        """The V-cycle's residual operator: FP64 -- K, or the matrix-free action."""
        if self.matrix_free:
            self.apply_matrix_free(x, y)
        else:
            self.spmv_exact(x, y)

    def apply_matrix_free(self, x, y):
        """y = K x for the Dirichlet-modified K: K(u) x, then y = x on the unit rows."""
        if self.mf_u is None and self.ev.kinematics != fcg.LINEAR:
            raise RuntimeError("matrix-free level: set_state(u) before the solve")
        self.ev.tangent_apply(self.mf_u, x, y, stream=self.stream())
        if self.mf_dbc.numel():
            y.index_copy_(0, self.mf_dbc, x.index_select(0, self.mf_dbc))


class _Indefinite(Exception):
    """The V-cycle returned a non-descent direction (r . z <= 0): smoother bound too low."""


class MultigridError(RuntimeError):
    """The preconditioned solve failed: with the kept lambda_max estimate and (Multigrid) again
    with a fresh one -- an indefinite V-cycle, or no convergence to the requested tolerance.  In
    the second case `iterations` and `relres` are set and x holds the last iterate, which a Newton
    loop with 'Rescue Bad Newton Solve' may still use as its direction."""

    def __init__(self, msg, iterations=None, relres=None):
        super().__init__(msg)
        self.iterations, self.relres = iterations, relres


class CycleFCG:
    """Flexible CG preconditioned by one V-cycle (the outer solve of Multigrid and amg.AMG).
    `retry_lmax`: on failure, re-estimate the fine level's lambda_max and solve once more (useful
    only where the estimate can be stale, i.e. Multigrid, which keeps it across tangents).
    Subclasses hold `levels` (level 0: the system's _Level on the evaluator's K) and supply
    _prepare(K) (per-tangent setup), _restrict(l, r, b_coarse), _prolong(l, x_coarse, x) (adds
    into x) and _coarse_solve(level, b, x); nu, ratio, boost, trace and dev as in Multigrid."""

    # post-smoothing on the finest level (False: the V-cycle pre-smooths only there -- a
    # nonsymmetric preconditioner, which the flexible CG's Polak-Ribiere beta admits; it saves
    # the fine level's two post-smoothing SpMVs of the five an iteration costs)
    fine_post = True
    retry_lmax = True

    # -- smoother ---------------------------------------------------------------------------
    # Chebyshev degree on the coarse levels (None: nu) and the cycle below the fine level
    # ("W": two coarse corrections per visit of a coarse level, which the cheap stencil levels
    # afford); the fine level is visited once per application either way
    coarse_nu = None
    cycle = "V"

    def _cheb(self, lvl, b, x, x_zero, nu=None):
        nu = self.nu if nu is None else nu
        lmax = self.boost * lvl.lmax
        lmin = lmax / self.ratio
        theta, delta = 0.5 * (lmax + lmin), 0.5 * (lmax - lmin)
        sigma = theta / delta
        rho = 1.0 / sigma
        r, d = lvl.r, lvl.d
        if getattr(lvl, "cheb_step", None) is not None and os.environ.get("FCG_MG_FUSED", "1") != "0":
            # the same steps, each update one fused pass (fcg_chebyshev_step), bit-identical
            if x_zero:
                lvl.cheb_step(b, None, d, x, 0.0, 1.0 / theta, 2)
            else:
                lvl.spmv(x, r)
                lvl.cheb_step(b, r, d, x, 0.0, 1.0 / theta, 0)
            for _ in range(nu - 1):
                lvl.spmv(x, r)
                rho_n = 1.0 / (2.0 * sigma - rho)
                lvl.cheb_step(b, r, d, x, rho_n * rho, 2.0 * rho_n / delta, 1)
                rho = rho_n
            return
        if x_zero:
            lvl.apply_dinv(b, d, 1.0 / theta)
            x.copy_(d)
        else:
            lvl.spmv(x, r)
            torch.sub(b, r, out=r)
            lvl.apply_dinv(r, d, 1.0 / theta)
            x.add_(d)
        for _ in range(nu - 1):
            lvl.spmv(x, r)
            torch.sub(b, r, out=r)
            rho_n = 1.0 / (2.0 * sigma - rho)
            d.mul_(rho_n * rho)
            lvl.apply_dinv(r, d, 2.0 * rho_n / delta, accumulate=True)
            x.add_(d)
            rho = rho_n

    def _vcycle(self, l, b, x):
        lvl = self.levels[l]
        if l == len(self.levels) - 1:
            self._coarse_solve(lvl, b, x)
            return
        nu = None if l == 0 or self.coarse_nu is None else self.coarse_nu
        self._cheb(lvl, b, x, x_zero=True, nu=nu)
        c = self.levels[l + 1]
        for _ in range(2 if l > 0 and self.cycle == "W" else 1):
            lvl.spmv_cycle(x, lvl.r)  # the restricted residual stays FP64 (mixed: smoother only)
            torch.sub(b, lvl.r, out=lvl.r)
            self._restrict(l, lvl.r, c.b)
            self._vcycle(l + 1, c.b, c.x)
            self._prolong(l, c.x, x)
        if l > 0 or self.fine_post:
            self._cheb(lvl, b, x, x_zero=False, nu=nu)

    # -- outer solve ------------------------------------------------------------------------
    def solve(self, K, b, x, rtol, max_iter=1000):
        """K x = b from x = 0 by flexible CG; returns (iterations, relative residual).

        A solve that meets an indefinite preconditioned step, or ends above rtol (a stale, too
        low lambda_max estimate lets the Chebyshev smoother amplify modes without r.z turning
        negative), re-estimates the fine level's lambda_max and restarts once; a second failure
        raises MultigridError."""
        f0 = self.levels[0]
        self._prepare(K)
        why, last = None, (None, None)
        for attempt in range(2 if self.retry_lmax else 1):
            if attempt:
                f0.estimate_lmax()
            try:
                it, rel = self._fcg(f0, b, x, rtol, max_iter)
            except (_Indefinite, FloatingPointError) as e:
                why, last = repr(e) or "indefinite V-cycle", (None, None)
                continue
            if rel <= rtol:
                return it, rel
            why, last = f"relative residual {rel:.3e} > {rtol:.3e} after {it} iterations", (it, rel)
        what = "after a lambda_max re-estimate" if self.retry_lmax else "(no retry)"
        raise MultigridError(f"multigrid FCG failed {what}: {why}", *last)

    # a V-cycle that never waits on the host (Multigrid with the dense coarsest solve) lets an
    # FCG iteration run as one captured HIP graph (FCG_MG_GRAPH=0: eager launches)
    graph_ok = False
    # the outer iteration's operator: the assembled K (default), or -- Multigrid with a
    # matrix-free fine level and outer_matrix_free=True -- the same Dirichlet-modified tangent
    # applied element by element (fcg_tangent_apply, = K x at 1e-13), 2.1 instead of 7.7 ms per
    # application at 1M hex27
    outer_matrix_free = False

    def _outer(self, f0, p, q):
        if self.outer_matrix_free:
            f0.apply_matrix_free(p, q)
        else:
            f0.spmv_exact(p, q)

    def _fcg(self, f0, b, x, rtol, max_iter):
        """Flexible CG with the scalars kept on the device: one host read per iteration (|r|,
        r.z and z.r_old together, after the V-cycle of the new residual -- the last iteration's
        V-cycle is spent for nothing, every other read would stall the queue)."""
        if self.graph_ok and os.environ.get("FCG_MG_GRAPH", "1") != "0" and not self.trace:
            return self._fcg_graph(f0, b, x, rtol, max_iter)
        if self.trace:
            print(f"  levels: {self.describe()}", file=sys.stderr, flush=True)
        bn = float(torch.linalg.vector_norm(b))
        x.zero_()
        if bn == 0.0:
            return 0, 0.0
        r = b.clone()
        z, q, r_old = (torch.empty_like(b) for _ in range(3))
        self._vcycle(0, r, z)
        p = z.clone()
        rz_t = torch.dot(r, z)
        rz = float(rz_t)
        if not rz > 0.0:
            raise _Indefinite()
        rn = bn
        it = 0
        while it < max_iter:
            it += 1
            self._outer(f0, p, q)
            alpha = rz_t / torch.dot(p, q)
            x.addcmul_(p, alpha)
            r_old.copy_(r)  # z . r_old enters the Polak-Ribiere beta
            r.addcmul_(q, alpha, value=-1.0)
            rr = torch.dot(r, r)
            self._vcycle(0, r, z)
            st = torch.stack((rr, torch.dot(r, z), torch.dot(z, r_old)))
            s3 = st.cpu().numpy()
            rn = float(np.sqrt(s3[0]))
            if not np.isfinite(rn):
                raise FloatingPointError("multigrid FCG diverged (non-finite residual)")
            if rn <= rtol * bn:
                break
            rz_new = float(s3[1])
            if not rz_new > 0.0:
                raise _Indefinite()
            beta = (rz_new - float(s3[2])) / rz
            if self.trace:
                print(f"  fcg {it}: |r|/|b| {rn / bn:.3e} rz {rz_new:.3e} beta {beta:.3e}",
                      file=sys.stderr, flush=True)
            p.mul_(beta).add_(z)
            rz, rz_t = rz_new, st[1]
        return it, rn / bn

    def _fcg_graph(self, f0, b, x, rtol, max_iter):
        """_fcg with one iteration -- the fine operator, the vector updates, the V-cycle and the
        dots, ~10^2 launches on 7 levels -- captured once into a HIP graph and replayed: the host
        launches one graph and reads |r|, r.z back per iteration, and the GPU no longer idles
        while Python issues the coarse levels' microsecond kernels.  alpha and the Polak-Ribiere
        beta stay device scalars.  The graph is rebuilt when what it baked in changes: the
        buffers of K, b, x, the state u of a matrix-free level, or a lambda_max."""
        bn = float(torch.linalg.vector_norm(b))
        x.zero_()
        if bn == 0.0:
            return 0, 0.0
        key = (b.data_ptr(), x.data_ptr(), b.numel(), f0.K.data_ptr(),
               None if f0.mf_u is None else f0.mf_u.data_ptr(),
               tuple(l.lmax for l in self.levels))
        g = getattr(self, "_graph", None)
        if g is None or g["key"] != key:
            f64 = dict(dtype=torch.float64, device=b.device)
            g = {"key": key, "graph": None}
            for name in ("r", "z", "q", "r_old", "p"):
                g[name] = torch.empty_like(b)
            for name in ("rz", "pq", "alpha", "beta", "rr", "rzn", "zro"):
                g[name] = torch.zeros((), **f64)
            g["st"] = torch.zeros(3, **f64)
            self._graph = g
        r, z, q, r_old, p = g["r"], g["z"], g["q"], g["r_old"], g["p"]

        def body():
            self._outer(f0, p, q)
            torch.dot(p, q, out=g["pq"])
            torch.div(g["rz"], g["pq"], out=g["alpha"])
            x.addcmul_(p, g["alpha"])
            r_old.copy_(r)  # z . r_old enters the Polak-Ribiere beta
            r.addcmul_(q, g["alpha"], value=-1.0)
            torch.dot(r, r, out=g["rr"])
            self._vcycle(0, r, z)
            torch.dot(r, z, out=g["rzn"])
            torch.dot(z, r_old, out=g["zro"])
            torch.div(g["rzn"] - g["zro"], g["rz"], out=g["beta"])
            p.mul_(g["beta"]).add_(z)
            g["rz"].copy_(g["rzn"])
            torch.stack((g["rr"], g["rzn"], g["zro"]), out=g["st"])

        r.copy_(b)
        self._vcycle(0, r, z)
        p.copy_(z)
        torch.dot(r, z, out=g["rz"])
        if not float(g["rz"]) > 0.0:
            raise _Indefinite()
        rn = bn
        it = 0
        while it < max_iter:
            it += 1
            if g["graph"] is not None:
                g["graph"].replay()
            else:
                body()  # the first iteration runs eagerly (warm-up), then the capture
                t_cap = time.perf_counter()
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph):
                    body()
                g["graph"] = graph
                if os.environ.get("FCG_MG_GRAPH_TIMING"):
                    print(f"  fcg graph captured in {1e3 * (time.perf_counter() - t_cap):.1f} ms",
                          file=sys.stderr, flush=True)
            s3 = g["st"].cpu().numpy()
            rn = float(np.sqrt(s3[0]))
            if not np.isfinite(rn):
                raise FloatingPointError("multigrid FCG diverged (non-finite residual)")
            if rn <= rtol * bn:
                break
            if not float(s3[1]) > 0.0:
                raise _Indefinite()
        return it, rn / bn


class Multigrid(CycleFCG):
    """Flexible-CG solver preconditioned by a geometric multigrid V-cycle (see module doc).

    fine_mesh / fine_ev: the discretisation being solved (BoxMesh + Evaluator, single rank);
    dbc_nodes(mesh) -> bool mask of the clamped nodes of a mesh of the same box (all 3 DOFs)."""

    def __init__(self, fine_mesh, fine_ev, dbc_nodes, youngs, poisson, nu=2, min_intervals=4,
                 max_levels=8, ratio=10.0, boost=1.1, coarse_rtol=1e-2, coarse_max_iter=2000,
                 mixed=False, coarse_solver="auto", fine_post=True, matrix_free=False,
                 outer_matrix_free=False):
        self.fine_post = bool(fine_post)
        if outer_matrix_free and not matrix_free:
            raise ValueError("outer_matrix_free needs the matrix-free fine level (matrix_free=True)")
        self.outer_matrix_free = bool(outer_matrix_free)
        if os.environ.get("FCG_MG_COARSE_NU"):
            self.coarse_nu = int(os.environ["FCG_MG_COARSE_NU"])
        if os.environ.get("FCG_MG_CYCLE"):
            self.cycle = os.environ["FCG_MG_CYCLE"]
        if matrix_free and (mixed or fine_mesh.celltype != fcg.HEX27):
            raise ValueError("matrix_free: hex27 fine levels in FP64 only (mixed=False)")
        if coarse_solver not in ("auto", "dense", "pcg", "amg"):
            raise ValueError(f"coarse_solver must be 'auto', 'dense', 'pcg' or 'amg', not {coarse_solver!r}")
        box = getattr(fine_mesh, "box", None)
        if box is None or getattr(fine_mesh, "nranks", 1) != 1:
            raise ValueError("Multigrid needs a single-rank GridGenerator box (fcg.BoxMesh)")
        iv = [int(box.interval[d]) for d in range(3)]
        meshes = []  # intervals of the hex8 coarse levels
        if fine_mesh.celltype == fcg.HEX27:
            meshes.append(tuple(iv))
        n = list(iv)
        # halve (odd counts to (n + 1) / 2, a non-nested level with general interpolation weights)
        while len(meshes) + 1 < max_levels and all((v + 1) // 2 >= min_intervals for v in n):
            n = [(v + 1) // 2 for v in n]
            meshes.append(tuple(n))
        if not meshes:
            raise ValueError(f"no coarse level for intervals {iv}: hex8 boxes need (n + 1) / 2 >= "
                             f"min_intervals ({min_intervals})")
        dev = torch.device("cuda", fine_ev.device)
        self.dev, self.nu, self.ratio, self.boost = dev, nu, ratio, boost
        # mixed: the fine level's Chebyshev smoother uses an FP32 copy of K (half the bytes of
        # 3 of the 5 SpMVs that dominate an iteration); the outer flexible CG and the restricted
        # residual keep the FP64 operator, so the solve still converges to the FP64 tolerance
        self.mixed = mixed
        self.coarse_rtol, self.coarse_max_iter = coarse_rtol, coarse_max_iter
        self.trace = bool(os.environ.get("FCG_MG_TRACE"))  # per-iteration residuals to stderr
        lower = [box.lower[d] for d in range(3)]
        upper = [box.upper[d] for d in range(3)]
        rot = [box.rotation[d] for d in range(3)]
        f64 = dict(dtype=torch.float64, device=dev)

        def dbc_rows(mesh):
            nodes = np.nonzero(dbc_nodes(mesh) & (mesh.node_dof_row >= 0))[0]
            return np.sort((mesh.node_dof_row[nodes][:, None] + np.arange(3)).ravel()).astype(np.int32)

        self.levels = [_Level(fine_mesh, fine_ev, None, dbc_rows(fine_mesh), dev)]
        self.levels[0].matrix_free = bool(matrix_free)
        if matrix_free:  # the action's per-context buffers and gather plan are set up here
            zc = torch.zeros(fine_mesh.n_cols, dtype=torch.float64, device=dev)
            fine_ev.tangent_apply(zc, zc, torch.empty(fine_mesh.n_rows, dtype=torch.float64, device=dev))
            del zc
        self.P, self.R, self.BT = [], [], []
        prev = fine_mesh
        tmr = bool(os.environ.get("FCG_MG_SETUP_TIMING"))
        for ivc in meshes:
            t_l = time.perf_counter()
            m = fcg.BoxMesh(fcg.HEX8, ivc, lower=lower, upper=upper, rotation=rot,
                            first_node_gid=int(box.first_node_gid))
            ev = fcg.Evaluator(m, kinematics=fcg.LINEAR, youngs=youngs, poisson=poisson,
                               device=fine_ev.device)
            K = torch.zeros(m.nnz, **f64)
            u0 = torch.zeros(m.n_cols, **f64)
            f0 = torch.zeros(m.n_rows, **f64)
            ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, u0, f0, K)
            rows = dbc_rows(m)
            ev.dirichlet_apply(torch.as_tensor(rows, device=dev), K)
            lvl = _Level(m, ev, K, rows, dev)
            lvl.setup_diag()
            # every element of a rediscretised box is the same parallelepiped: the level applies
            # its 27-point stencil instead of reading K (FCG_MG_STENCIL=0: the assembled K)
            if os.environ.get("FCG_MG_STENCIL", "1") != "0" and min(ivc) >= 1:
                lvl.stencil = box_stencil(m, youngs, poisson, dev, rows)
            # a 2:1 pair (hex27 -> hex8 on the same elements, hex8 n -> n/2): weights implicit
            # (FCG_MG_BOXT=0: the tables); the node-block tables only where that does not apply
            # (at 1M hex27 they took most of this setup's time, unused)
            bt = None
            if os.environ.get("FCG_MG_BOXT", "1") != "0":
                try:
                    bt = _BoxTransfer(prev, self.levels[-1].rows, m, rows, dev)
                except ValueError:
                    bt = None
            self.BT.append(bt)
            if bt is None:
                P, R = transfer_tables(prev, m)
                self.P.append(_Transfer(P, dev))
                self.R.append(_Transfer(R, dev))
            else:
                self.P.append(None)
                self.R.append(None)
            self.levels.append(lvl)
            prev = m
            if tmr:
                torch.cuda.synchronize()
                print(f"  multigrid level {ivc}: {time.perf_counter() - t_l:.2f} s", file=sys.stderr, flush=True)
        t_l = time.perf_counter()
        for lvl in self.levels[1:-1]:
            lvl.estimate_lmax()
        if tmr:
            print(f"  multigrid lambda_max estimates: {time.perf_counter() - t_l:.2f} s", file=sys.stderr, flush=True)
        # coarsest level: its rediscretised linear operator does not change between tangents, so
        # it is factored once -- "dense": the inverse of the (small) matrix, one matrix-vector
        # product per V-cycle, exact and without the host round trips of an iterative solve;
        # "pcg": block-Jacobi PCG to coarse_rtol (fcg_pcg_solve); "amg": the native
        # smoothed-aggregation AMG set up on it.  "auto": dense up to 6,000 DOFs, else PCG.
        self.coarse_amg = None
        self.coarse_inv = None
        last = self.levels[-1]
        if coarse_solver == "auto":
            coarse_solver = "dense" if last.n <= 6000 else "pcg"
        self.coarse_solver = coarse_solver
        self.graph_ok = coarse_solver == "dense"  # the V-cycle never waits on the host
        if coarse_solver == "dense":
            Kh = last.K.cpu().numpy()
            A = np.zeros((last.n, last.n))
            rows = np.repeat(np.arange(last.n), np.diff(last.mesh.rowptr))
            A[rows, last.mesh.col_lid] = Kh
            self.coarse_inv = torch.from_numpy(np.linalg.inv(A)).to(dev)
        if coarse_solver == "amg":
            from .amg import NativeAMG
            last = self.levels[-1]
            self.coarse_amg = NativeAMG(last.mesh, last.ev, last.rows)
            self.coarse_amg.setup(last.K)

    def warm_up(self):
        """Launch every kernel of a solve once on scratch data, so that the first Newton step
        does not pay the process's one-time costs (HIP loads a kernel's code object at its first
        launch; config 3's first solve took ~0.3 s longer than the others).  Keeps no state: the
        fine level's lambda_max stays unestimated, its block inverses are recomputed by the next
        solve's _prepare, no graph is captured."""
        f0 = self.levels[0]
        f64 = dict(dtype=torch.float64, device=self.dev)
        saved = (f0.lmax, f0.mf_u)
        f0.dinv.zero_()
        f0.lmax = 1.0
        if f0.matrix_free:
            f0.mf_u = torch.zeros(f0.mesh.n_cols, **f64)
        try:
            b = torch.zeros(f0.n, **f64)
            x = torch.zeros(f0.n, **f64)
            self._vcycle(0, b, x)
            if self.outer_matrix_free:
                self._outer(f0, b, x)
            sc = torch.zeros((), **f64)
            torch.dot(b, x, out=sc)
            torch.div(sc, sc + 1.0, out=sc)
            x.addcmul_(b, sc)
            x.mul_(sc).add_(b)
            st = torch.zeros(3, **f64)
            torch.stack((sc, sc, sc), out=st)
            st.cpu()
            float(torch.linalg.vector_norm(b))
        finally:
            f0.lmax, f0.mf_u = saved
        torch.cuda.synchronize(self.dev)

    def describe(self):
        out = [{"celltype": "hex27" if l.mesh.celltype == fcg.HEX27 else "hex8",
                "intervals": [int(l.mesh.box.interval[d]) for d in range(3)], "dofs": l.n,
                "lmax": l.lmax} for l in self.levels]
        out[-1]["coarse_solver"] = self.coarse_solver
        if self.levels[0].matrix_free:
            out[0]["operator"] = "matrix-free (fcg_tangent_apply)"
            out[0]["outer_operator"] = "matrix-free" if self.outer_matrix_free else "assembled K"
        return out

    def set_state(self, u_col):
        """The displacement the next solve's tangent was evaluated at (the matrix-free fine
        level applies K(u); StaticNewton calls this before each linear solve)."""
        self.levels[0].mf_u = u_col

    def _prepare(self, K):
        """lambda_max of D^-1 K barely moves between Newton iterations: it is estimated on the
        first solve and kept (re-estimated by CycleFCG.solve's restart)."""
        t0 = time.perf_counter()
        f0 = self.levels[0]
        f0.K = K
        if self.mixed:
            if f0.K32 is None or f0.K32.numel() != K.numel():
                f0.K32 = torch.empty(K.numel(), dtype=torch.float32, device=K.device)
            f0.K32.copy_(K)
        f0.setup_diag()
        if f0.lmax is None:
            f0.estimate_lmax()
            if os.environ.get("FCG_MG_GRAPH_TIMING"):
                print(f"  fine lambda_max estimate {1e3 * (time.perf_counter() - t0):.1f} ms",
                      file=sys.stderr, flush=True)

    def _restrict(self, l, r, cb):
        if self.BT[l] is not None:
            self.BT[l].restrict(r, cb)
            return
        self.R[l](r, cb, accumulate=False)
        cb.mul_(self.levels[l + 1].mask)

    def _prolong(self, l, cx, x):
        if self.BT[l] is not None:
            self.BT[l].prolong(cx, x)
            return
        self.P[l](cx, x, accumulate=True)
        x.mul_(self.levels[l].mask)

    def _coarse_solve(self, lvl, b, x):
        if self.coarse_inv is not None:
            torch.mv(self.coarse_inv, b, out=x)
            return
        if self.coarse_amg is not None:
            self.coarse_amg.solve(lvl.K, b, x, self.coarse_rtol, self.coarse_max_iter, setup=False)
            return
        lvl.ev.pcg_solve(lvl.K, b, x, self.coarse_rtol, self.coarse_max_iter,
                         stream=torch.cuda.current_stream(self.dev))

    # -- outer solve ------------------------------------------------------------------------
    def check_dirichlet(self, dbc_rows):
        """The fine level's mask (from dbc_nodes) must constrain exactly the Newton's Dirichlet
        rows, else prolongation leaves values on constrained rows that the unit rows never
        correct; raises ValueError when the two sets differ."""
        mine = np.sort(self.levels[0].rows)
        theirs = np.sort(np.asarray(dbc_rows, dtype=np.int32))
        if not np.array_equal(mine, theirs):
            raise ValueError(f"multigrid Dirichlet rows ({len(mine)}) differ from the system's "
                             f"({len(theirs)}): pass a dbc_nodes mask with the same nodes and all "
                             f"three DOFs constrained")
