"""Multi-GPU bindings (ctypes) of the library's RCCL data path, include/fourc_gpu.h "Multi-GPU":

  Comm          fcg_comm: one RCCL communicator per rank (id from rank 0 through any host channel)
  ImportPlan    fcg_import_plan_build: Discretization::set_state's row -> column import
                (4C_fem_discretization.cpp:503-548), built on the host with one exchange callback
  Halo          fcg_halo_*: the import on device buffers -- RCCL grouped send / recv
                (`import_`) or the pack / unpack halves around a host transport
  SharedPlan    fcg_shared_plan_build: the interface of a strict element partition
  Shared        fcg_shared_*: the shared-DOF residual all-reduce (SURVEY §8e option B)
  residual_norm fcg_norm2: ||f|| over the ranks (NOX's Norm2 -> MPI_Allreduce)

The exchange callback (`fcg_alltoallv_fn`) is an MPI_Alltoallv in a 4C host; here it is either
the RCCL one of a Comm (`comm.exchange`) or `gloo_exchange()` over torch.distributed (tests and
host-staged rehearsals on CPU or on one GPU shared by several ranks).  The product path moves no
data through Python: every evaluate-time byte moves in the library.
"""

import ctypes
import importlib

import numpy as np

fcg = importlib.import_module("4c_amd.fcg")
_i32p, _i64p, _dp = fcg._i32p, fcg._i64p, fcg._dp


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _stream(stream, device):
    return fcg._torch_stream(stream, device)


class Comm:
    """fcg_comm over RCCL.  `bcast_id(bytes_or_None) -> bytes` delivers rank 0's id to every rank
    (a TCPStore, MPI_Bcast, ...)."""

    def __init__(self, rank, world, device, bcast_id):
        L = fcg.lib()
        buf = (ctypes.c_char * 128)()
        if rank == 0:
            rc = L.fcg_comm_unique_id(buf)
            if rc != 0:
                raise fcg.FcgError(rc, "fcg_comm_unique_id failed")
            uid = bcast_id(bytes(buf))
        else:
            uid = bcast_id(None)
        ctypes.memmove(buf, uid, 128)
        h = ctypes.c_void_p()
        # RCCL prints its version banner on stdout at init: send it to stderr, so that a host's
        # stdout (bench.py's one JSON line) stays clean
        import os
        import sys
        sys.stdout.flush()
        saved = os.dup(1)
        try:
            os.dup2(2, 1)
            rc = L.fcg_comm_create(buf, world, rank, device, ctypes.byref(h))
        finally:
            os.dup2(saved, 1)
            os.close(saved)
        if rc != 0:
            raise fcg.FcgError(rc, "fcg_comm_create (ncclCommInitRank) failed")
        self._h, self.rank, self.world, self.device = h, rank, world, device
        self.exchange = Exchange(ctypes.cast(L.fcg_comm_alltoallv, ctypes.c_void_p).value, h)

    def size(self):
        """ncclCommCount of the communicator (fcg_comm_size)."""
        n = ctypes.c_int()
        rc = fcg.lib().fcg_comm_size(self._h, ctypes.byref(n))
        if rc != 0:
            raise fcg.FcgError(rc, "fcg_comm_size failed")
        return n.value

    def allreduce(self, t, op=fcg.FCG_OP_SUM, stream=None):
        """In-place all-reduce of a float64 device tensor."""
        rc = fcg.lib().fcg_comm_allreduce(self._h, _ptr(t), t.numel(), op,
                                          _stream(stream, self.device))
        if rc != 0:
            raise fcg.FcgError(rc, "fcg_comm_allreduce failed")

    def close(self):
        if getattr(self, "_h", None):
            fcg.lib().fcg_comm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Exchange:
    """An fcg_alltoallv_fn plus its user pointer."""

    def __init__(self, fn_addr, user, keepalive=None):
        self.fn = fcg.ALLTOALLV_FN(fn_addr) if isinstance(fn_addr, int) else fn_addr
        self.user = user
        self._keep = keepalive


def gloo_exchange():
    """fcg_alltoallv_fn over torch.distributed (CPU tensors; gloo).  Exceptions become a non-zero
    return, which the library reports as FCG_ERR_DEVICE."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size()

    def cb(send, scounts, recv, rcounts, item, _user):
        try:
            sc = [int(scounts[p]) * item for p in range(world)]
            rcn = [int(rcounts[p]) * item for p in range(world)]
            sbuf = torch.empty(sum(sc), dtype=torch.uint8)
            if sum(sc):
                ctypes.memmove(sbuf.data_ptr(), send, sum(sc))
            rbuf = torch.empty(sum(rcn), dtype=torch.uint8)
            dist.all_to_all_single(rbuf, sbuf, output_split_sizes=rcn, input_split_sizes=sc)
            if sum(rcn):
                ctypes.memmove(recv, rbuf.data_ptr(), sum(rcn))
            return 0
        except Exception:  # noqa: BLE001 - surfaced as an error code
            return 1

    fn = fcg.ALLTOALLV_FN(cb)
    return Exchange(fn, None, keepalive=cb)


def thread_exchanges(world, timeout=None, barrier_out=None):
    """`world` fcg_alltoallv_fn callbacks for ranks that are threads of ONE process (MPI_Alltoallv
    semantics through shared memory and a barrier): plan builds of every rank of a partition
    from one process -- a host that evaluates the ranks of a split in turn on one device, and the
    CPU tests.  Rank r's plan build must run in its own thread with exchanges[r] (`run_ranks`).
    `timeout` (s) bounds every barrier wait; `barrier_out` (a list) receives the barrier, so that
    a caller can abort it when a rank fails outside its exchanges."""
    import threading
    barrier = threading.Barrier(world, timeout=timeout)
    if barrier_out is not None:
        barrier_out.append(barrier)
    slots = [None] * world
    out = []
    for rank in range(world):
        def cb(send, scounts, recv, rcounts, item, _user, rank=rank):
            try:
                sc = [int(scounts[p]) for p in range(world)]
                total = sum(sc) * item
                slots[rank] = (ctypes.string_at(send, total) if total else b"", sc)
                barrier.wait()
                off = 0
                for p in range(world):
                    buf, psc = slots[p]
                    start, n = sum(psc[:rank]) * item, psc[rank] * item
                    if n != int(rcounts[p]) * item:
                        raise ValueError("alltoallv: send and receive counts disagree")
                    if n:
                        ctypes.memmove(recv + off, buf[start:start + n], n)
                    off += n
                barrier.wait()  # every rank has read the slots before any rank reuses its own
                return 0
            except Exception:  # noqa: BLE001 - surfaced as an error code
                barrier.abort()
                return 1

        fn = fcg.ALLTOALLV_FN(cb)
        out.append(Exchange(fn, None, keepalive=cb))
    return out


def run_ranks(world, fn, timeout=600.0):
    """fn(rank, exchange) for every rank, each in its own thread over thread_exchanges(world);
    returns the results in rank order (re-raises the first failure).  A rank that raises (or
    calls its exchange a different number of times than the others) aborts the shared barrier, so
    the other ranks fail instead of waiting forever; every wait is bounded by `timeout` seconds."""
    import threading
    bar = []
    xs = thread_exchanges(world, timeout=timeout, barrier_out=bar)
    res, err = [None] * world, [None] * world

    def body(r):
        try:
            res[r] = fn(r, xs[r])
        except BaseException as e:  # noqa: BLE001 - re-raised in the caller
            err[r] = e
            bar[0].abort()

    ts = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for e in err:
        if e is not None:
            raise e
    return res


def _arr(p, n, dt):
    if n == 0:
        return np.zeros(0, dtype=dt)
    return np.ctypeslib.as_array(p, shape=(n,)).astype(dt, copy=True)


class ImportPlan:
    """fcg_import_plan_build on the rank's maps (collective over the exchange)."""

    def __init__(self, rank, world, row_gid, col_gid, col_owner, exchange):
        row_gid = np.ascontiguousarray(row_gid, dtype=np.int32)
        col_gid = np.ascontiguousarray(col_gid, dtype=np.int32)
        col_owner = np.ascontiguousarray(col_owner, dtype=np.int32)
        plan, store = fcg.FcgImportPlan(), ctypes.c_void_p()
        rc = fcg.lib().fcg_import_plan_build(
            rank, world, len(row_gid), row_gid.ctypes.data_as(_i32p), len(col_gid),
            col_gid.ctypes.data_as(_i32p), col_owner.ctypes.data_as(_i32p), exchange.fn,
            exchange.user, ctypes.byref(plan), ctypes.byref(store))
        if rc != 0:
            raise fcg.FcgError(rc, "fcg_import_plan_build failed")
        self._plan, self._store = plan, store
        self.n_same, self.n_permute = plan.n_same, plan.n_permute
        self.permute_from = _arr(plan.permute_from, plan.n_permute, np.int32)
        self.permute_to = _arr(plan.permute_to, plan.n_permute, np.int32)
        self.send_counts = _arr(plan.send_counts, world, np.int64)
        self.recv_counts = _arr(plan.recv_counts, world, np.int64)
        self.send_row = _arr(plan.send_row, int(self.send_counts.sum()), np.int32)
        self.recv_col = _arr(plan.recv_col, int(self.recv_counts.sum()), np.int32)

    @classmethod
    def from_arrays(cls, rank, world, n_rows, n_cols, n_same, permute_from, permute_to,
                    send_counts, send_row, recv_counts, recv_col):
        """An explicit plan (e.g. the lists of an existing Epetra_Import), no exchange."""
        self = cls.__new__(cls)
        self._store = None
        a = dict(permute_from=np.ascontiguousarray(permute_from, dtype=np.int32),
                 permute_to=np.ascontiguousarray(permute_to, dtype=np.int32),
                 send_counts=np.ascontiguousarray(send_counts, dtype=np.int64),
                 send_row=np.ascontiguousarray(send_row, dtype=np.int32),
                 recv_counts=np.ascontiguousarray(recv_counts, dtype=np.int64),
                 recv_col=np.ascontiguousarray(recv_col, dtype=np.int32))
        plan = fcg.FcgImportPlan()
        plan.nranks, plan.rank, plan.n_rows, plan.n_cols = world, rank, n_rows, n_cols
        plan.n_same, plan.n_permute = n_same, len(a["permute_from"])
        for k, v in a.items():
            setattr(plan, k, v.ctypes.data_as(_i64p if v.dtype == np.int64 else _i32p))
            setattr(self, k, v)
        self._plan, self.n_same, self.n_permute = plan, n_same, plan.n_permute
        return self

    def apply_host(self, u_row, u_col, recv):
        """Host restatement of pack + unpack (for tests): returns the send buffer and fills the
        owned and ghost columns from u_row and the received values."""
        u_col[:self.n_same] = u_row[:self.n_same]
        u_col[self.permute_to] = u_row[self.permute_from]
        if recv is not None:
            u_col[self.recv_col] = recv
        return u_row[self.send_row]

    def close(self):
        if getattr(self, "_store", None):
            fcg.lib().fcg_plan_free(self._store)
            self._store = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Halo:
    """fcg_halo on `device` for an ImportPlan."""

    def __init__(self, plan, device):
        h = ctypes.c_void_p()
        rc = fcg.lib().fcg_halo_create(ctypes.byref(plan._plan), device, ctypes.byref(h))
        if rc != 0:
            raise fcg.FcgError(rc, "fcg_halo_create failed")
        self._h, self.device = h, device
        self.n_send = int(plan.send_counts.sum())
        self.n_recv = int(plan.recv_counts.sum())
        self.send_counts, self.recv_counts = plan.send_counts.tolist(), plan.recv_counts.tolist()

    def import_(self, comm, u_row, u_col, stream=None):
        """set_state over RCCL (asynchronous on the stream)."""
        rc = fcg.lib().fcg_halo_import(self._h, comm._h, _ptr(u_row), _ptr(u_col),
                                       _stream(stream, self.device))
        if rc != 0:
            raise fcg.FcgError(rc, "fcg_halo_import failed")

    def pack(self, u_row, u_col, send, stream=None):
        rc = fcg.lib().fcg_halo_pack(self._h, _ptr(u_row), _ptr(u_col), _ptr(send),
                                     _stream(stream, self.device))
        if rc != 0:
            raise fcg.FcgError(rc, "fcg_halo_pack failed")

    def unpack(self, recv, u_col, stream=None):
        rc = fcg.lib().fcg_halo_unpack(self._h, _ptr(recv), _ptr(u_col), _stream(stream, self.device))
        if rc != 0:
            raise fcg.FcgError(rc, "fcg_halo_unpack failed")

    def import_staged(self, u_row, u_col, stream=None):
        """Host-staged transport over torch.distributed (gloo): pack on the device, move the
        bytes through the host, unpack on the device (several ranks on one GPU, MPI-style hosts)."""
        import torch
        import torch.distributed as dist
        send = torch.empty(max(1, self.n_send), dtype=torch.float64, device=u_row.device)
        self.pack(u_row, u_col, send, stream)
        (stream or torch.cuda.current_stream(u_row.device)).synchronize()
        rb = torch.empty(self.n_recv, dtype=torch.float64)
        dist.all_to_all_single(rb, send[:self.n_send].cpu(), output_split_sizes=self.recv_counts,
                               input_split_sizes=self.send_counts)
        # the device copy of the received values is made on `stream`, the stream unpack is queued
        # on, and both buffers are marked in use by it, so that the caching allocator cannot hand
        # them to other work before unpack has run
        st = stream or torch.cuda.current_stream(u_row.device)
        with torch.cuda.stream(st):
            recv = rb.to(u_row.device, non_blocking=False)
        recv.record_stream(st)
        send.record_stream(st)
        self.unpack(recv, u_col, st)

    def close(self):
        if getattr(self, "_h", None):
            fcg.lib().fcg_halo_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class SharedPlan:
    """fcg_shared_plan_build for a strict BoxMesh rank (or any rank with owned + extended rows)."""

    def __init__(self, rank, world, owned_gid, ext_gid, ext_owner, exchange):
        owned_gid = np.ascontiguousarray(owned_gid, dtype=np.int32)
        ext_gid = np.ascontiguousarray(ext_gid, dtype=np.int32)
        ext_owner = np.ascontiguousarray(ext_owner, dtype=np.int32)
        plan, store = fcg.FcgSharedPlan(), ctypes.c_void_p()
        rc = fcg.lib().fcg_shared_plan_build(
            rank, world, len(owned_gid), owned_gid.ctypes.data_as(_i32p), len(ext_gid),
            ext_gid.ctypes.data_as(_i32p), ext_owner.ctypes.data_as(_i32p), exchange.fn,
            exchange.user, ctypes.byref(plan), ctypes.byref(store))
        if rc != 0:
            raise fcg.FcgError(rc, "fcg_shared_plan_build failed")
        self._plan, self._store = plan, store
        self.n_global, self.n_owned = plan.n_global, plan.n_owned
        self.row = _arr(plan.row, plan.n_local, np.int32)
        self.pos = _arr(plan.pos, plan.n_local, np.int64)

    @classmethod
    def from_arrays(cls, rank, world, n_global, n_owned, row, pos):
        self = cls.__new__(cls)
        self._store = None
        self.row = np.ascontiguousarray(row, dtype=np.int32)
        self.pos = np.ascontiguousarray(pos, dtype=np.int64)
        plan = fcg.FcgSharedPlan()
        plan.nranks, plan.rank, plan.n_global = world, rank, n_global
        plan.n_local, plan.n_owned = len(self.row), n_owned
        plan.row, plan.pos = self.row.ctypes.data_as(_i32p), self.pos.ctypes.data_as(_i64p)
        self._plan, self.n_global, self.n_owned = plan, n_global, n_owned
        return self

    @staticmethod
    def of_mesh(mesh, exchange):
        """The plan of a strict BoxMesh rank: extended rows are the column DOFs past the owned
        rows, owned by their node's owner."""
        n_own = mesh.n_owned_rows
        owner = col_owner_of(mesh)
        return SharedPlan(mesh.rank, mesh.nranks, mesh.row_gid[:n_own], mesh.row_gid[n_own:],
                          owner[n_own:], exchange)

    def pack_host(self, f):
        buf = np.zeros(self.n_global)
        buf[self.pos] = f[self.row]
        return buf

    def unpack_host(self, buf, f):
        f[self.row[:self.n_owned]] = buf[self.pos[:self.n_owned]]

    def close(self):
        if getattr(self, "_store", None):
            fcg.lib().fcg_plan_free(self._store)
            self._store = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Shared:
    """fcg_shared on `device`."""

    def __init__(self, plan, device):
        h = ctypes.c_void_p()
        rc = fcg.lib().fcg_shared_create(ctypes.byref(plan._plan), device, ctypes.byref(h))
        if rc != 0:
            raise fcg.FcgError(rc, "fcg_shared_create failed")
        self._h, self.device, self.n_global = h, device, plan.n_global

    def reduce(self, comm, f, stream=None):
        rc = fcg.lib().fcg_shared_reduce(self._h, comm._h, _ptr(f), _stream(stream, self.device))
        if rc != 0:
            raise fcg.FcgError(rc, "fcg_shared_reduce failed")

    def pack(self, f, buf, stream=None):
        rc = fcg.lib().fcg_shared_pack(self._h, _ptr(f), _ptr(buf), _stream(stream, self.device))
        if rc != 0:
            raise fcg.FcgError(rc, "fcg_shared_pack failed")

    def unpack(self, buf, f, stream=None):
        rc = fcg.lib().fcg_shared_unpack(self._h, _ptr(buf), _ptr(f), _stream(stream, self.device))
        if rc != 0:
            raise fcg.FcgError(rc, "fcg_shared_unpack failed")

    def reduce_staged(self, f, stream=None):
        """Host-staged transport (gloo all-reduce of the interface buffer)."""
        import torch
        import torch.distributed as dist
        st = stream or torch.cuda.current_stream(f.device)
        with torch.cuda.stream(st):
            buf = torch.empty(max(1, self.n_global), dtype=torch.float64, device=f.device)
            self.pack(f, buf, st)
            h = buf[:self.n_global].cpu()
            dist.all_reduce(h)
            buf[:self.n_global].copy_(h)
            self.unpack(buf, f, st)

    def close(self):
        if getattr(self, "_h", None):
            fcg.lib().fcg_shared_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def col_owner_of(mesh):
    """Owning rank of every column DOF of a BoxMesh rank."""
    owner = np.empty(mesh.n_cols, dtype=np.int32)
    for d in range(3):
        owner[mesh.node_dof_col + d] = mesh.node_owner
    return owner


def residual_norm(f_row, comm=None, stream=None):
    """fcg_norm2: ||f|| over all ranks of `comm` (this rank only without one); blocking."""
    out = ctypes.c_double()
    rc = fcg.lib().fcg_norm2(comm._h if comm is not None else None, _ptr(f_row), f_row.numel(),
                             _stream(stream, f_row.device), ctypes.byref(out))
    if rc != 0:
        raise fcg.FcgError(rc, "fcg_norm2 failed")
    return out.value
