"""World-size 2 / 4 gloo tests of the multi-rank path on CPU.  The library's host
plan builders (fcg_import_plan_build, fcg_shared_plan_build) run in every rank and exchange
through gloo; the data movement the device kernels do (pack / RCCL / unpack) is restated on the
host from the plan arrays, and the CPU oracle evaluates every rank's elements:

* option A (the reference's semantics, 4C_fem_discretization.cpp:542-548 + owned rows only):
  set_state's import reproduces the global column vector, and halo + evaluate gives every rank
  exactly the global K and f_int rows it owns;
* option B (north_star's shared-DOF all-reduce): strict element partition, each rank's partial
  f_int summed over the interface buffer, equals the global f_int on the owned rows;
* the residual norm over ranks equals the global norm.
"""

import importlib
import os
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _setup(rank, world, port):
    for p in (ROOT, os.path.join(ROOT, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    fcg = importlib.import_module("4c_amd").fcg
    halo = importlib.import_module("4c_amd.halo")
    return fcg, halo


def _global_state(fcg, celltype, iv, kinem, amp):
    from parity_util import oracle_evaluate
    glob = fcg.BoxMesh(celltype, iv, jitter=0.1, seed=20251015)
    ug = glob.u_col(amp)
    err, _, Kg, fg = oracle_evaluate(glob, kinem, 210.0, 0.3, ug)
    assert err == 0
    return glob, ug, Kg, fg


def _worker_option_a(rank, world, port, q, celltype, iv, kinem):
    try:
        fcg, halo = _setup(rank, world, port)
        from parity_util import oracle_evaluate
        amp = 1e-3 if kinem == fcg.LINEAR else 5e-2
        glob, ug, Kg, fg = _global_state(fcg, celltype, iv, kinem, amp)
        gcol = {int(g): i for i, g in enumerate(glob.col_gid)}
        m = fcg.BoxMesh(celltype, iv, jitter=0.1, seed=20251015, rank=rank, nranks=world)
        plan = halo.ImportPlan(rank, world, m.row_gid, m.col_gid, halo.col_owner_of(m),
                               halo.gloo_exchange())
        # Epetra column layout: owned prefix, then per owner one contiguous ghost block
        assert plan.n_same == m.n_rows and plan.n_permute == 0
        off = 0
        for p in range(world):
            c = plan.recv_col[off:off + plan.recv_counts[p]]
            assert np.array_equal(c, np.arange(c[0], c[0] + len(c))) if len(c) else True
            off += plan.recv_counts[p]
        u_row = np.array([ug[gcol[int(g)]] for g in m.row_gid])
        u_col = np.full(m.n_cols, np.nan)
        send = plan.apply_host(u_row, u_col, None)
        recv = torch.empty(int(plan.recv_counts.sum()), dtype=torch.float64)
        dist.all_to_all_single(recv, torch.from_numpy(np.ascontiguousarray(send)),
                               output_split_sizes=plan.recv_counts.tolist(),
                               input_split_sizes=plan.send_counts.tolist())
        plan.apply_host(u_row, u_col, recv.numpy())
        expect = np.array([ug[gcol[int(g)]] for g in m.col_gid])
        ok_import = np.array_equal(u_col, expect)
        # halo + evaluate: the rank's owned rows equal the global rows
        err, _, K, f = oracle_evaluate(m, kinem, 210.0, 0.3, u_col)
        grow = {int(g): i for i, g in enumerate(glob.row_gid)}
        gi = np.array([grow[int(g)] for g in m.row_gid])
        df = np.abs(f - fg[gi]).max() / np.abs(fg).max()
        # K rows: compare (row gid, col gid) -> value
        dK = 0.0
        for r in range(m.n_rows):
            a, b = m.rowptr[r], m.rowptr[r + 1]
            ga, gb = glob.rowptr[gi[r]], glob.rowptr[gi[r] + 1]
            # local columns are sorted by LID (Epetra), so compare entries keyed by column GID
            cols = m.col_gid[m.col_lid[a:b]]
            gcols = glob.col_gid[glob.col_lid[ga:gb]]
            o, go = np.argsort(cols), np.argsort(gcols)
            assert np.array_equal(cols[o], gcols[go])  # same (row GID, col GID) set, bit-exact
            dK = max(dK, np.abs(K[a:b][o] - Kg[ga:gb][go]).max())
        dK /= np.abs(Kg).max()
        q.put((rank, bool(ok_import) and err == 0, float(df), float(dK), int(plan.recv_counts.sum())))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, traceback.format_exc() + repr(e), 1.0, 1.0, -1))


def _worker_option_b(rank, world, port, q, celltype, iv, kinem):
    try:
        fcg, halo = _setup(rank, world, port)
        from parity_util import oracle_evaluate
        amp = 1e-3 if kinem == fcg.LINEAR else 5e-2
        glob, ug, _, fg = _global_state(fcg, celltype, iv, kinem, amp)
        gcol = {int(g): i for i, g in enumerate(glob.col_gid)}
        grow = {int(g): i for i, g in enumerate(glob.row_gid)}
        m = fcg.BoxMesh(celltype, iv, jitter=0.1, seed=20251015, rank=rank, nranks=world,
                        strict=True)
        assert m.n_ele == m.n_ele_row  # strict: no ghost elements
        assert m.n_rows == m.n_cols and np.array_equal(m.row_gid, m.col_gid)
        # the strict rank needs u on every node of its row elements: the import of its map
        plan = halo.ImportPlan(rank, world, m.row_gid[:m.n_owned_rows], m.col_gid,
                               halo.col_owner_of(m), halo.gloo_exchange())
        u_col = np.array([ug[gcol[int(g)]] for g in m.col_gid])
        err, _, _, f = oracle_evaluate(m, kinem, 210.0, 0.3, u_col, want_k=False)
        sp = halo.SharedPlan.of_mesh(m, halo.gloo_exchange())
        buf = torch.from_numpy(sp.pack_host(f))
        dist.all_reduce(buf)
        sp.unpack_host(buf.numpy(), f)
        own = f[:m.n_owned_rows]
        gi = np.array([grow[int(g)] for g in m.row_gid[:m.n_owned_rows]])
        rel = float(np.linalg.norm(own - fg[gi]) / np.linalg.norm(fg[gi]))
        nrm = float(np.linalg.norm(own) ** 2)
        t = torch.tensor([nrm], dtype=torch.float64)
        dist.all_reduce(t)
        q.put((rank, err == 0 and plan.n_permute == 0, rel, sp.n_global,
               float(np.sqrt(t.item()) / np.linalg.norm(fg) - 1.0)))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, traceback.format_exc() + repr(e), 1.0, -1, 1.0))


def _spawn(target, world, args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + world * 7 + os.getpid() % 1000 + hash(target.__name__) % 97
    procs = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    return res


@pytest.mark.parametrize("world,celltype,kinem", [(2, 0, 0), (4, 0, 1), (2, 1, 1)])
def test_option_a_halo_evaluate(world, celltype, kinem):
    iv = (6, 5, 4) if celltype == 0 else (3, 2, 2)
    for rank, ok, df, dK, nrecv in _spawn(_worker_option_a, world, (celltype, iv, kinem)):
        assert ok is True, (rank, ok)
        assert nrecv > 0
        assert df <= 1e-12 and dK <= 1e-12, (rank, df, dK)


@pytest.mark.parametrize("world,celltype,kinem", [(2, 0, 0), (4, 0, 1), (8, 0, 0), (2, 1, 0)])
def test_option_b_shared_allreduce(world, celltype, kinem):
    iv = (6, 6, 4) if celltype == 0 else (3, 2, 2)
    res = _spawn(_worker_option_b, world, (celltype, iv, kinem))
    n_globals = {r[3] for r in res}
    assert len(n_globals) == 1 and next(iter(n_globals)) > 0  # one buffer shared by all ranks
    for rank, ok, rel, _, dn in res:
        assert ok is True, (rank, ok)
        assert rel <= 1e-12, (rank, rel)
        assert abs(dn) <= 1e-12


@pytest.mark.parametrize("world", [2, 8])
def test_thread_exchange_plans_match_the_global_maps(world):
    """halo.run_ranks: the plan builds of every rank of a split from ONE process (ranks as threads,
    fcg_alltoallv_fn through shared memory) -- how the config-4 GPU test builds the 8 ranks'
    plans.  The import reproduces every rank's column vector and the shared-DOF reduce of the
    strict ranks' oracle partials gives the global f_int on the owned rows."""
    fcg = importlib.import_module("4c_amd").fcg
    halo = importlib.import_module("4c_amd.halo")
    from parity_util import oracle_evaluate
    iv = (6, 6, 4)
    glob, ug, _, fg = _global_state(fcg, 0, iv, 0, 1e-3)
    gcol = {int(g): i for i, g in enumerate(glob.col_gid)}
    grow = {int(g): i for i, g in enumerate(glob.row_gid)}
    meshes = [fcg.BoxMesh(0, iv, jitter=0.1, seed=20251015, rank=r, nranks=world) for r in range(world)]
    plans = halo.run_ranks(world, lambda r, x: halo.ImportPlan(
        r, world, meshes[r].row_gid, meshes[r].col_gid, halo.col_owner_of(meshes[r]), x))
    u_rows = [np.array([ug[gcol[int(g)]] for g in m.row_gid]) for m in meshes]
    sends = [plans[r].apply_host(u_rows[r], np.empty(meshes[r].n_cols), None) for r in range(world)]
    for r, m in enumerate(meshes):
        # peer p's segment for r sits after p's segments for ranks < r
        recv = np.concatenate([sends[p][int(plans[p].send_counts[:r].sum()):
                                        int(plans[p].send_counts[:r + 1].sum())] for p in range(world)])
        u_col = np.full(m.n_cols, np.nan)
        plans[r].apply_host(u_rows[r], u_col, recv)
        assert np.array_equal(u_col, np.array([ug[gcol[int(g)]] for g in m.col_gid])), r
    strict = [fcg.BoxMesh(0, iv, jitter=0.1, seed=20251015, rank=r, nranks=world, strict=True)
              for r in range(world)]
    sps = halo.run_ranks(world, lambda r, x: halo.SharedPlan.of_mesh(strict[r], x))
    assert len({p.n_global for p in sps}) == 1
    parts = []
    for r, m in enumerate(strict):
        u = np.array([ug[gcol[int(g)]] for g in m.col_gid])
        err, _, _, f = oracle_evaluate(m, 0, 210.0, 0.3, u, want_k=False)
        assert err == 0
        parts.append(f)
    total = sum(sps[r].pack_host(parts[r]) for r in range(world))
    for r, m in enumerate(strict):
        sps[r].unpack_host(total, parts[r])
        own = parts[r][:m.n_owned_rows]
        gi = np.array([grow[int(g)] for g in m.row_gid[:m.n_owned_rows]])
        assert np.abs(own - fg[gi]).max() <= 1e-12 * np.abs(fg).max(), r


def test_run_ranks_fails_instead_of_hanging_when_a_rank_raises():
    """A rank that raises before its exchange aborts the shared barrier: the other rank's plan
    build fails (its exchange returns an error code) and run_ranks re-raises, no hang."""
    import time
    fcg = importlib.import_module("4c_amd").fcg
    halo = importlib.import_module("4c_amd.halo")
    world = 2
    meshes = [fcg.BoxMesh(0, (4, 2, 2), rank=r, nranks=world) for r in range(world)]

    def fn(r, x):
        if r == 1:
            time.sleep(0.2)  # rank 0 is already waiting in its exchange
            raise ValueError("rank 1 failed before its exchange")
        return halo.ImportPlan(r, world, meshes[r].row_gid, meshes[r].col_gid,
                               halo.col_owner_of(meshes[r]), x)

    t0 = time.time()
    with pytest.raises(Exception):
        halo.run_ranks(world, fn, timeout=60.0)
    assert time.time() - t0 < 30.0
