"""Multi-rank linear solve and static Newton over the C-ABI halo (SURVEY §8f row 2 across ranks).

4C hands the distributed Epetra tangent to Belos CG with a point-block relaxation preconditioner
(`4C_solver_nonlin_nox_linearsystem.cpp:275-353`; Ifpack point-block Jacobi, local to each rank)
and NOX's full Newton measures the residual with Epetra `Norm2` (local sum + MPI_Allreduce).  Here
every rank holds the owned rows of K in its column-map CSR (what `fcg_evaluate_device` assembles
with the ghost-layer partition, option A):

* the operator K p needs p in the column map: `fcg_halo_import` (RCCL grouped send/recv, or
  host-staged through gloo) imports the ghost entries before `fcg_spmv`, as
  `Epetra_CrsMatrix::Multiply` imports through the matrix's Importer;
* the preconditioner is the inverse of the 3 x 3 nodal diagonal blocks of the owned rows
  (`fcg_block_jacobi_setup` / `apply`), no communication;
* dot products are local sums combined by one all-reduce of two numbers per iteration.

`DistributedNewton` is `newton.StaticNewton` across ranks: set_state import of the displacement
into the column map, evaluate, r = f_int - f_ext, Dirichlet rows, the global residual norm,
`DistributedPCG` for the increment.  Transport: an RCCL `halo.Comm`, or None with `staged=True`
(host-staged halo + gloo sums: several ranks on one device, where RCCL refuses)."""

import ctypes
import importlib

import numpy as np
import torch
import torch.distributed as dist

fcg = importlib.import_module("4c_amd").fcg
halo = importlib.import_module("4c_amd.halo")
newton = importlib.import_module("4c_amd.newton")


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


class Transport:
    """Halo import and all-reduce of a few float64 numbers, over RCCL or host-staged gloo."""

    def __init__(self, imp, comm=None, staged=False, device=0):
        self.imp, self.comm, self.staged = imp, comm, staged
        self.dev = torch.device("cuda", device)
        if not staged and comm is None:
            raise ValueError("Transport needs an RCCL halo.Comm unless staged=True")

    def import_(self, x_row, x_col, stream=None):
        if self.staged:
            self.imp.import_staged(x_row, x_col, stream)
        else:
            self.imp.import_(self.comm, x_row, x_col, stream)

    def sum(self, vals):
        """Sum of the ranks' `vals` (a float64 device tensor), returned as a host numpy array."""
        if self.staged:
            t = vals.cpu()
            if dist.is_initialized() and dist.get_world_size() > 1:
                dist.all_reduce(t)
            return t.numpy()
        self.comm.allreduce(vals)
        return vals.cpu().numpy()


class DistributedPCG:
    """Preconditioned CG on the ranks' owned rows: solve(K, b, x, rtol, max_iter) ->
    (iterations, relative residual), x = 0 start, |r| <= rtol |b| over all ranks (the
    `StaticNewton` linear-solver interface)."""

    def __init__(self, evaluator, transport):
        info = evaluator.info
        self.ev, self.tr = evaluator, transport
        self.n, self.n_cols = int(info.n_rows), int(info.n_cols)
        self.dev = torch.device("cuda", evaluator.device)
        f64 = dict(dtype=torch.float64, device=self.dev)
        self.r = torch.empty(self.n, **f64)
        self.z = torch.empty(self.n, **f64)
        self.p = torch.empty(self.n, **f64)
        self.q = torch.empty(self.n, **f64)
        self.p_col = torch.zeros(self.n_cols, **f64)
        self.dinv = torch.empty(3 * self.n, **f64)  # 3 x 3 inverse per node (9 per 3 rows)
        self.iterations, self.rel_residual = 0, None

    def _precond(self, r, z):
        s = torch.cuda.current_stream(self.dev).cuda_stream
        rc = fcg.lib().fcg_block_jacobi_apply(self.ev._h, _ptr(self.dinv), _ptr(r), _ptr(z), 1.0, 0,
                                              ctypes.c_void_p(s))
        if rc != 0:
            raise fcg.FcgError(rc, fcg.lib().fcg_last_error(self.ev._h).decode())

    def _op(self, K, p, q):
        self.tr.import_(p, self.p_col)
        self.ev.spmv(K, self.p_col, q)

    def solve(self, K, b, x, rtol=1e-10, max_iter=10000):
        s = torch.cuda.current_stream(self.dev).cuda_stream
        rc = fcg.lib().fcg_block_jacobi_setup(self.ev._h, _ptr(K), _ptr(self.dinv), ctypes.c_void_p(s))
        if rc != 0:
            raise fcg.FcgError(rc, fcg.lib().fcg_last_error(self.ev._h).decode())
        x.zero_()
        self.r.copy_(b)
        self._precond(self.r, self.z)
        self.p.copy_(self.z)
        two = torch.empty(2, dtype=torch.float64, device=self.dev)
        two[0] = torch.dot(self.r, self.z)
        two[1] = torch.dot(b, b)
        rz, bb = self.tr.sum(two)
        bn = float(np.sqrt(bb))
        if bn == 0.0:
            self.iterations, self.rel_residual = 0, 0.0
            return 0, 0.0
        rn = bn
        it = 0
        while it < max_iter:
            self._op(K, self.p, self.q)
            pq = float(self.tr.sum(torch.dot(self.p, self.q).reshape(1))[0])
            if not (pq > 0.0):
                raise fcg.FcgError(fcg.FCG_ERR_SINGULAR, f"PCG breakdown: p.Kp = {pq} at iteration {it}")
            alpha = rz / pq
            x.add_(self.p, alpha=alpha)
            self.r.add_(self.q, alpha=-alpha)
            it += 1
            self._precond(self.r, self.z)
            two[0] = torch.dot(self.r, self.z)
            two[1] = torch.dot(self.r, self.r)
            rz_new, rr = self.tr.sum(two)
            rn = float(np.sqrt(rr))
            if not np.isfinite(rn):
                raise fcg.FcgError(fcg.FCG_ERR_SINGULAR, "PCG: non-finite residual")
            if rn <= rtol * bn:
                break
            self.p.mul_(rz_new / rz).add_(self.z)
            rz = rz_new
        self.iterations, self.rel_residual = it, rn / bn
        return it, rn / bn


class NativeDFCG:
    """fcg_dfcg_solve: the same distributed solve as one native call (fcg_dsolve.hip) -- flexible
    CG with one import per SpMV and all-reduced inner products, preconditioned by the rank's
    NativeAMG on its owned block (amg) or the nodal block Jacobi (amg=None).  `transport`:
    a Transport over RCCL (halo.Comm) or host-staged (gloo callbacks into the library).  Same
    solve(K, b, x, rtol, max_iter) interface as DistributedPCG."""

    def __init__(self, evaluator, transport, amg=None, coupled=True):
        """coupled=False: the transport does not name the ranks (nranks = 0), so the AMG stays the
        rank-local subdomain preconditioner (the round-3 behaviour, kept for comparison)."""
        self.ev, self.tr, self.amg = evaluator, transport, amg
        self.dev = torch.device("cuda", evaluator.device)
        self._keep = []
        L = fcg.lib()
        t = fcg.FcgTransport()
        if not transport.staged:
            self._pair = fcg.FcgRcclPair(transport.comm._h.value, transport.imp._h.value)
            rc = L.fcg_transport_rccl(ctypes.byref(self._pair), ctypes.byref(t))
            if rc != 0:
                raise fcg.FcgError(rc, "fcg_transport_rccl failed")
        else:
            imp = transport.imp
            send = torch.empty(max(1, imp.n_send), dtype=torch.float64, device=self.dev)
            recv = torch.empty(max(1, imp.n_recv), dtype=torch.float64, device=self.dev)

            def import_cb(_user, x_row, x_col, stream):
                try:
                    Lb = fcg.lib()
                    rc = Lb.fcg_halo_pack(imp._h, x_row, x_col, _ptr(send), stream)
                    if rc != 0:
                        return rc
                    torch.cuda.synchronize(self.dev)
                    rb = torch.empty(imp.n_recv, dtype=torch.float64)
                    dist.all_to_all_single(rb, send[:imp.n_send].cpu(), output_split_sizes=imp.recv_counts,
                                           input_split_sizes=imp.send_counts)
                    recv[:imp.n_recv].copy_(rb)
                    torch.cuda.synchronize(self.dev)
                    return Lb.fcg_halo_unpack(imp._h, _ptr(recv), x_col, stream)
                except Exception:  # noqa: BLE001 - surfaced as an error code
                    return fcg.FCG_ERR_DEVICE

            def allreduce_cb(_user, d_vals, n, _stream):
                try:
                    Lb = fcg.lib()
                    h = np.zeros(n)
                    if Lb.fcg_memcpy_d2h(h.ctypes.data_as(ctypes.c_void_p), d_vals, 8 * n) != 0:
                        return fcg.FCG_ERR_DEVICE
                    ht = torch.from_numpy(h)
                    if dist.is_initialized() and dist.get_world_size() > 1:
                        dist.all_reduce(ht)
                    return Lb.fcg_memcpy_h2d(d_vals, ht.numpy().ctypes.data_as(ctypes.c_void_p), 8 * n)
                except Exception:  # noqa: BLE001
                    return fcg.FCG_ERR_DEVICE

            def exchange_cb(_user, d_send, scnt, d_recv, rcnt, _stream):
                # the distributed coarse level's point-to-point exchange: MPI_Alltoallv of doubles
                try:
                    Lb = fcg.lib()
                    world = dist.get_world_size()
                    sc = [int(scnt[q]) for q in range(world)]
                    rc = [int(rcnt[q]) for q in range(world)]
                    torch.cuda.synchronize(self.dev)
                    hs = np.zeros(max(1, sum(sc)))
                    if sum(sc) and Lb.fcg_memcpy_d2h(hs.ctypes.data_as(ctypes.c_void_p), d_send, 8 * sum(sc)) != 0:
                        return fcg.FCG_ERR_DEVICE
                    hr = torch.empty(sum(rc), dtype=torch.float64)
                    dist.all_to_all_single(hr, torch.from_numpy(hs[:sum(sc)]), output_split_sizes=rc,
                                           input_split_sizes=sc)
                    if sum(rc):
                        return Lb.fcg_memcpy_h2d(d_recv, hr.numpy().ctypes.data_as(ctypes.c_void_p), 8 * sum(rc))
                    return 0
                except Exception:  # noqa: BLE001 - surfaced as an error code
                    return fcg.FCG_ERR_DEVICE

            t.import_fn = fcg.IMPORT_FN(import_cb)
            t.allreduce_fn = fcg.ALLREDUCE_FN(allreduce_cb)
            t.exchange_fn = fcg.EXCHANGE_FN(exchange_cb)
            self._keep += [t.import_fn, t.allreduce_fn, t.exchange_fn, send, recv]
            if dist.is_initialized():
                t.rank, t.nranks = dist.get_rank(), dist.get_world_size()
            else:
                t.rank, t.nranks = 0, 1
        if not coupled:
            t.nranks = 0
        self._t = t
        self.iterations, self.rel_residual = 0, None

    def solve(self, K, b, x, rtol=1e-10, max_iter=10000):
        it, rel = ctypes.c_int(0), ctypes.c_double(0.0)
        s = ctypes.c_void_p(torch.cuda.current_stream(self.dev).cuda_stream)
        rc = fcg.lib().fcg_dfcg_solve(self.ev._h, self.amg._h if self.amg is not None else None,
                                      ctypes.byref(self._t), _ptr(K), _ptr(b), _ptr(x), float(rtol),
                                      int(max_iter), s, ctypes.byref(it), ctypes.byref(rel))
        if rc != 0:
            raise fcg.FcgError(rc, fcg.lib().fcg_last_error(self.ev._h).decode())
        self.iterations, self.rel_residual = it.value, rel.value
        return it.value, rel.value

    def coupled_levels(self):
        """Levels of the AMG hierarchy coupled across ranks (0: rank-local preconditioner)."""
        return fcg.lib().fcg_amg_coupled_levels(self.amg._h) if self.amg is not None else 0

    COUPLED_STATS = ("distributed_levels", "level1_rows_here", "level1_rows_global",
                     "allreduce_doubles_setup", "allreduce_doubles_apply", "exchange_doubles_setup",
                     "exchange_doubles_apply", "replicated_bytes", "replicated_rows")

    def coupled_stats(self):
        """fcg_amg_coupled_stats: what the coupled coarse levels store and move on this rank."""
        if self.amg is None:
            return {}
        out = (ctypes.c_int64 * len(self.COUPLED_STATS))()
        n = fcg.lib().fcg_amg_coupled_stats(self.amg._h, out, len(self.COUPLED_STATS))
        return {k: int(out[i]) for i, k in enumerate(self.COUPLED_STATS[:max(0, n)])}


class DistributedNewton:
    """Static full Newton on the ranks of a ghost-layer partition: the rank's Evaluator (its
    column elements, owned rows), the halo Transport, the owned rows' external force and
    Dirichlet row LIDs.  solve() returns the converged owned-row displacement."""

    def __init__(self, evaluator, transport, fext_row, dbc_rows, tol_res=1e-10, tol_inc=1e-10,
                 max_iter=20, lin_rtol=1e-12, lin_max_iter=100000, rescue_bad_newton_solve=True,
                 linear_solver=None):
        info = evaluator.info
        self.ev, self.tr = evaluator, transport
        self.dev = torch.device("cuda", evaluator.device)
        self.n, self.n_cols, self.nnz = int(info.n_rows), int(info.n_cols), int(info.nnz)
        f64 = dict(dtype=torch.float64, device=self.dev)
        self.fext = torch.as_tensor(np.asarray(fext_row, dtype=np.float64)).to(self.dev)
        self.dbc = torch.as_tensor(np.asarray(dbc_rows, dtype=np.int32)).to(self.dev)
        self.K = torch.empty(self.nnz, **f64)
        self.fint = torch.empty(self.n, **f64)
        self.r = torch.empty(self.n, **f64)
        self.du = torch.empty(self.n, **f64)
        self.u_col = torch.zeros(self.n_cols, **f64)
        self.freact = torch.zeros(self.n, **f64)
        self.tol_res, self.tol_inc, self.max_iter = tol_res, tol_inc, max_iter
        self.lin_rtol, self.lin_max_iter = lin_rtol, lin_max_iter
        self.rescue = rescue_bad_newton_solve  # NOX "Rescue Bad Newton Solve" (newton.StaticNewton)
        # linear_solver: e.g. NativeDFCG (the native solve with a rank-local AMG); default the
        # block-Jacobi DistributedPCG
        self.pcg = linear_solver if linear_solver is not None else DistributedPCG(evaluator, transport)
        self.history = []

    def _norm(self, v):
        return float(np.sqrt(self.tr.sum(torch.dot(v, v).reshape(1))[0]))

    def solve(self, u0=None):
        u = (torch.zeros(self.n, dtype=torch.float64, device=self.dev) if u0 is None
             else torch.as_tensor(u0, dtype=torch.float64).to(self.dev).clone())
        self.history = []
        ndu = float("inf")
        for it in range(self.max_iter + 1):
            self.tr.import_(u, self.u_col)                      # set_state
            self.ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, self.u_col, self.fint, self.K)
            torch.sub(self.fint, self.fext, out=self.r)
            self.ev.dirichlet_apply(self.dbc, self.K, self.r, self.freact)
            nr = self._norm(self.r)
            rec = {"iter": it, "norm_res": nr, "norm_inc": ndu if it else None}
            if it > 0 and nr <= self.tol_res and ndu <= self.tol_inc:
                self.history.append(rec)
                return u
            torch.neg(self.r, out=self.r)
            lin_it, lin_res = newton.accept_linear_solve(
                lambda: self.pcg.solve(self.K, self.r, self.du, self.lin_rtol, self.lin_max_iter),
                self.lin_rtol, it, self.rescue, rec)
            rec.update(lin_iter=lin_it, lin_relres=lin_res)
            self.history.append(rec)
            ndu = self._norm(self.du)
            u += self.du
            if nr == 0.0 and ndu == 0.0:
                return u
        raise RuntimeError(f"Newton did not converge in {self.max_iter} iterations: {self.history[-3:]}")
