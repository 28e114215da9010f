"""GPU tests of the multi-GPU data path through the C ABI.

RCCL refuses two ranks on one device, so on a one-GPU box:
* the RCCL entry points run on a one-rank communicator: fcg_halo_import with an explicit plan
  whose peer is the rank itself (grouped ncclSend / ncclRecv loopback, contiguous and scattered
  ghost blocks), fcg_comm_allreduce, fcg_norm2 and fcg_shared_reduce;
* the multi-rank steps run as two processes on the GPU with the library's pack / unpack halves
  around a host-staged gloo transport, and are compared with the CPU oracle:
  option A (ghost layer: halo import + evaluate, owned rows == the global rows) and option B
  (strict element partition: evaluate + shared-DOF all-reduce, owned rows == the global f_int).
"""

import importlib
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
torch = pytest.importorskip("torch")
fcg = importlib.import_module("4c_amd").fcg
halo = importlib.import_module("4c_amd.halo")

pytestmark = pytest.mark.gpu

E, NU = 210.0, 0.3


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _comm1():
    return halo.Comm(0, 1, 0, lambda b: b)


@pytest.mark.parametrize("contiguous", [True, False])
def test_rccl_loopback_halo_import(contiguous):
    dev = _dev()
    comm = _comm1()
    rng = np.random.default_rng(3)
    n_rows, k = 200, 57
    n_cols = n_rows + k + 5
    perm_to = np.arange(n_rows, n_rows + 5)
    perm_from = rng.choice(n_rows, 5, replace=False)
    send_row = rng.choice(n_rows, k, replace=False)
    recv_col = np.arange(n_rows + 5, n_cols)
    if not contiguous:
        recv_col = rng.permutation(recv_col)
    plan = halo.ImportPlan.from_arrays(0, 1, n_rows, n_cols, n_rows, perm_from, perm_to, [k],
                                       send_row, [k], recv_col)
    h = halo.Halo(plan, 0)
    u_row = torch.from_numpy(rng.standard_normal(n_rows)).to(dev)
    u_col = torch.full((n_cols,), float("nan"), dtype=torch.float64, device=dev)
    for _ in range(3):  # repeated imports reuse the library's buffers
        h.import_(comm, u_row, u_col)
    torch.cuda.synchronize()
    ur = u_row.cpu().numpy()
    expect = np.empty(n_cols)
    expect[:n_rows] = ur
    expect[perm_to] = ur[perm_from]
    expect[recv_col] = ur[send_row]
    assert np.array_equal(u_col.cpu().numpy(), expect)
    h.close()
    comm.close()


def test_rccl_allreduce_norm_and_shared_single_rank():
    dev = _dev()
    comm = _comm1()
    x = torch.from_numpy(np.random.default_rng(4).standard_normal(1_000_003)).to(dev)
    y = x.clone()
    comm.allreduce(y)
    comm.allreduce(y, op=fcg.FCG_OP_MAX)
    torch.cuda.synchronize()
    assert torch.equal(x, y)
    ref = float(np.linalg.norm(x.cpu().numpy()))
    for c in (comm, None):
        n = halo.residual_norm(x, c)
        assert abs(n - ref) <= 1e-13 * ref
        assert n == halo.residual_norm(x, c)  # fixed summation order: bitwise repeatable
    # shared reduce on one rank: the owned interface rows get the buffer values back
    f = torch.from_numpy(np.arange(10, dtype=np.float64)).to(dev)
    sp = halo.SharedPlan.from_arrays(0, 1, 6, 3, [1, 4, 7, 0, 2, 9], [5, 0, 2, 1, 3, 4])
    s = halo.Shared(sp, 0)
    s.reduce(comm, f)
    torch.cuda.synchronize()
    assert np.array_equal(f.cpu().numpy(), np.arange(10, dtype=np.float64))
    s.close()
    comm.close()


def test_async_evaluate_defers_errors():
    """fcg_set_async: the failing evaluate returns at once; fcg_check_error reports 4C's throw
    with the element GID, and the context recovers for the next evaluate."""
    dev = _dev()
    mesh = fcg.BoxMesh(fcg.HEX8, (2, 2, 2))
    good = fcg.BoxMesh(fcg.HEX8, (2, 2, 2))
    mesh.node_x[:, 0] *= -1.0
    ev = fcg.Evaluator(mesh, kinematics=fcg.LINEAR, youngs=E, poisson=NU)
    ev.set_async(True)
    u = torch.zeros(mesh.n_cols, dtype=torch.float64, device=dev)
    f = torch.zeros(mesh.n_rows, dtype=torch.float64, device=dev)
    K = torch.zeros(mesh.nnz, dtype=torch.float64, device=dev)
    ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, u, f, K)  # queued, no error yet
    ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, u, f, K)  # sticky until checked
    with pytest.raises(fcg.FcgError) as ei:
        ev.check_error()
    assert ei.value.code == 1 and ei.value.bad_ele_gid == 0
    ev.check_error()  # nothing pending any more
    ev2 = fcg.Evaluator(good, kinematics=fcg.LINEAR, youngs=E, poisson=NU)
    ev2.set_async(True)
    ev2.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, u, f, K)
    ev2.check_error()
    ev2.set_async(False)


def test_async_element_error_survives_dirichlet_and_solver():
    """The Newton order of INTEGRATION.md: evaluate (async) -> fcg_dirichlet_apply -> the solve's
    block-Jacobi setup -> fcg_check_error.  The Dirichlet and solver kernels report through their
    own flag word, so the failed element's flag (4C's throw) is still there when checked."""
    dev = _dev()
    mesh = fcg.BoxMesh(fcg.HEX8, (2, 2, 2))
    mesh.node_x[:, 0] *= -1.0
    ev = fcg.Evaluator(mesh, kinematics=fcg.LINEAR, youngs=E, poisson=NU)
    ev.set_async(True)
    u = torch.zeros(mesh.n_cols, dtype=torch.float64, device=dev)
    f = torch.zeros(mesh.n_rows, dtype=torch.float64, device=dev)
    K = torch.zeros(mesh.nnz, dtype=torch.float64, device=dev)
    ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, u, f, K)
    rows = torch.arange(0, 6, dtype=torch.int32, device=dev)
    ev.dirichlet_apply(rows, K, f.clone())
    with pytest.raises(fcg.FcgError) as ei:
        ev.check_error()
    assert ei.value.code == 1 and ei.value.bad_ele_gid == 0
    ev.set_async(False)


@pytest.mark.parametrize("threads", ["8", "0"])
def test_host_overwrite_entry_point(threads):
    """fcg_evaluate_host(OVERWRITE): the caller's zero() fused -- garbage in K and f is
    overwritten, the result equals the oracle; ACCUMULATE adds (fcg_evaluate)."""
    from parity_util import oracle_evaluate, rel_err
    _dev()
    os.environ["FCG_HOST_COPY_THREADS"] = threads
    mesh = fcg.BoxMesh(fcg.HEX8, (12, 10, 9), jitter=0.1)
    u = mesh.u_col(1e-3)
    ev = fcg.Evaluator(mesh, kinematics=fcg.LINEAR, youngs=E, poisson=NU)
    K = np.full(mesh.nnz, 7.0)
    f = np.full(mesh.n_rows, -3.0)
    ev.evaluate_host(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, u, f, K)
    _, _, Kr, fr = oracle_evaluate(mesh, fcg.LINEAR, E, NU, u)
    assert rel_err(f, fr) <= 1e-10 and rel_err(K, Kr) <= 1e-12
    ev.evaluate_host(fcg.CALC_NLNSTIFF, fcg.ACCUMULATE, u, f, K)
    assert rel_err(f, 2 * fr) <= 1e-10 and rel_err(K, 2 * Kr) <= 1e-12


# ------------------------------------------------------------------ two ranks, host-staged
def _worker(rank, world, port, q, option, celltype, kinem, path):
    try:
        for p in (ROOT, os.path.join(ROOT, "tests")):
            if p not in sys.path:
                sys.path.insert(0, p)
        import torch.distributed as dist
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from parity_util import oracle_evaluate, rel_err
        dev = torch.device("cuda:0")
        iv = (8, 6, 5) if celltype == fcg.HEX8 else (3, 3, 2)
        amp = 1e-3 if kinem == fcg.LINEAR else 5e-2
        glob = fcg.BoxMesh(celltype, iv, jitter=0.1 if celltype == fcg.HEX8 else 0.02, seed=5)
        ug = glob.u_col(amp)
        gcol = {int(g): i for i, g in enumerate(glob.col_gid)}
        strict = option == "B"
        m = fcg.BoxMesh(celltype, iv, jitter=0.1 if celltype == fcg.HEX8 else 0.02, seed=5,
                        rank=rank, nranks=world, strict=strict)
        n_own = m.n_owned_rows
        plan = halo.ImportPlan(rank, world, m.row_gid[:n_own], m.col_gid, halo.col_owner_of(m),
                               halo.gloo_exchange())
        h = halo.Halo(plan, 0)
        u_row = torch.from_numpy(np.array([ug[gcol[int(g)]] for g in m.row_gid[:n_own]])).to(dev)
        u_col = torch.full((m.n_cols,), float("nan"), dtype=torch.float64, device=dev)
        h.import_staged(u_row, u_col)
        torch.cuda.synchronize()
        u_exp = np.array([ug[gcol[int(g)]] for g in m.col_gid])
        ok = bool(np.array_equal(u_col.cpu().numpy(), u_exp))
        ev = fcg.Evaluator(m, kinematics=kinem, youngs=E, poisson=NU, device=0, path=path)
        ev.set_async(True)
        f = torch.full((m.n_rows,), float("nan"), dtype=torch.float64, device=dev)
        out = {"path": ev.info.path}
        if option == "A":
            K = torch.full((m.nnz,), float("nan"), dtype=torch.float64, device=dev)
            ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, u_col, f, K)
            ev.check_error()
            _, _, Kr, fr = oracle_evaluate(m, kinem, E, NU, u_exp)
            Kg = K.cpu().numpy()
            out["dK"] = float(rel_err(Kg, Kr))
            out["dKmax"] = float(np.abs(Kg - Kr).max() / np.abs(Kr).max())
            out["df"] = float(rel_err(f.cpu().numpy(), fr))
            fg_own = fr
        else:
            ev.evaluate_device(fcg.CALC_INTERNALFORCE, fcg.OVERWRITE, u_col, f)
            ev.check_error()
            sh = halo.Shared(halo.SharedPlan.of_mesh(m, halo.gloo_exchange()), 0)
            sh.reduce_staged(f)
            torch.cuda.synchronize()
            _, _, _, fgl = oracle_evaluate(glob, kinem, E, NU, ug, want_k=False)
            grow = {int(g): i for i, g in enumerate(glob.row_gid)}
            fg_own = fgl[[grow[int(g)] for g in m.row_gid[:n_own]]]
            out["df"] = float(rel_err(f[:n_own].cpu().numpy(), fg_own))
            out["n_global"] = sh.n_global
        # residual norm over the ranks (fcg_norm2 locally, the sum of squares through gloo)
        loc = halo.residual_norm(f[:n_own])
        t = torch.tensor([loc * loc], dtype=torch.float64)
        dist.all_reduce(t)
        ref = torch.tensor([float(np.dot(fg_own, fg_own))], dtype=torch.float64)
        dist.all_reduce(ref)
        out["dnorm"] = abs(np.sqrt(t.item()) - np.sqrt(ref.item())) / np.sqrt(ref.item())
        q.put((rank, ok, out))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, traceback.format_exc() + repr(e), {}))


def _spawn(world, args):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29600 + os.getpid() % 1000 + world
    procs = [ctx.Process(target=_worker, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    return res


@pytest.mark.parametrize("celltype,kinem,path", [
    (fcg.HEX8, fcg.LINEAR, fcg.PATH_AUTO), (fcg.HEX8, fcg.TOTLAG, fcg.PATH_GENERAL),
    (fcg.HEX27, fcg.TOTLAG, fcg.PATH_AUTO)])
def test_two_ranks_option_a_halo_evaluate(celltype, kinem, path):
    _dev()
    for rank, ok, out in _spawn(2, ("A", celltype, kinem, path)):
        assert ok is True, (rank, ok)
        assert out["df"] <= 1e-10 and out["dK"] <= 1e-12 and out["dKmax"] <= 1e-12, (rank, out)
        assert out["dnorm"] <= 1e-10


@pytest.mark.parametrize("celltype,kinem,path", [
    (fcg.HEX8, fcg.LINEAR, fcg.PATH_AUTO), (fcg.HEX8, fcg.LINEAR, fcg.PATH_GENERAL),
    (fcg.HEX8, fcg.TOTLAG, fcg.PATH_AUTO), (fcg.HEX27, fcg.LINEAR, fcg.PATH_GENERAL)])
def test_two_ranks_option_b_shared_allreduce(celltype, kinem, path):
    _dev()
    res = _spawn(2, ("B", celltype, kinem, path))
    assert res[0][2].get("n_global") == res[1][2].get("n_global") and res[0][2]["n_global"] > 0
    for rank, ok, out in res:
        assert ok is True, (rank, ok)
        if celltype == fcg.HEX8 and path == fcg.PATH_AUTO:
            assert out["path"] == fcg.PATH_STRUCTURED  # strict ranks keep the fused sweep
        assert out["df"] <= 1e-10, (rank, out)
        assert out["dnorm"] <= 1e-10


# ------------------------------------------------------ multi-rank Newton + PCG (host-staged)
def _cantilever_loads(m, x_max):
    """x = 0 clamped (all DOFs of the rank's owned nodes there), -1e-3 in z on every owned node at
    x = x_max (point loads by GID: the same on any partition)."""
    X = m.node_x
    own = m.node_dof_row >= 0
    fext = np.zeros(m.n_rows)
    tip = np.nonzero(own & np.isclose(X[:, 0], x_max))[0]
    for nd in tip:
        fext[m.node_dof_row[nd] + 2] = -1e-3
    cl = np.nonzero(own & np.isclose(X[:, 0], 0.0))[0]
    dbc = np.sort((m.node_dof_row[cl][:, None] + np.arange(3)).ravel()).astype(np.int32)
    return fext, dbc


def _worker_solve(rank, world, port, q, kinem, path, transport="staged", solver="pcg",
                  celltype=None):
    try:
        for p in (ROOT, os.path.join(ROOT, "tests")):
            if p not in sys.path:
                sys.path.insert(0, p)
        import torch.distributed as dist
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dsolve = importlib.import_module("4c_amd.dsolve")
        ct = fcg.HEX8 if celltype is None else celltype
        iv, up = _solve_box(ct)
        m = fcg.BoxMesh(ct, iv, upper=up, jitter=0.1 if ct == fcg.HEX8 else 0.02, seed=5, rank=rank,
                        nranks=world)
        n_own = m.n_owned_rows
        comm = None
        if transport == "rccl":  # one GPU per rank: halo + dots over the library's RCCL comm
            dev = rank
            torch.cuda.set_device(dev)

            def bcast(b):
                box = [b]
                dist.broadcast_object_list(box, src=0)
                return box[0]
            comm = halo.Comm(rank, world, dev, bcast)
            xchg = comm.exchange
        else:
            dev, xchg = 0, halo.gloo_exchange()
        plan = halo.ImportPlan(rank, world, m.row_gid[:n_own], m.col_gid, halo.col_owner_of(m), xchg)
        h = halo.Halo(plan, dev)
        ev = fcg.Evaluator(m, kinematics=kinem, youngs=E, poisson=NU, device=dev, path=path)
        fext, dbc = _cantilever_loads(m, up[0])
        tr = (dsolve.Transport(h, comm=comm, device=dev) if comm is not None
              else dsolve.Transport(h, staged=True, device=dev))
        lin = None
        if solver != "pcg":
            amg_mod = importlib.import_module("4c_amd.amg")
            amg = amg_mod.NativeAMG(m, ev, dbc) if solver in ("native", "native-uncoupled") else None
            lin = dsolve.NativeDFCG(ev, tr, amg, coupled=solver != "native-uncoupled")
        nt = dsolve.DistributedNewton(ev, tr, fext, dbc, tol_res=1e-10, tol_inc=1e-11, lin_rtol=1e-12,
                                      linear_solver=lin)
        u = nt.solve().cpu().numpy()
        q.put((rank, True, {"u": dict(zip(m.row_gid[:n_own].tolist(), u.tolist())),
                            "iters": [r.get("lin_iter") for r in nt.history],
                            "coupled_levels": lin.coupled_levels() if lin is not None else 0,
                            "stats": lin.coupled_stats() if lin is not None else {}}))
        if lin is not None and lin.amg is not None:
            lin.amg.close()
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, traceback.format_exc() + repr(e), {}))


def _solve_box(celltype):
    box = os.environ.get("FCG_TEST_SOLVE_BOX")  # "nx,ny,nz": a larger hex8 box for the stats tests
    if box and celltype == fcg.HEX8:
        n = tuple(int(v) for v in box.split(","))
        return n, tuple(float(v) for v in n)
    return ((8, 4, 4), (8.0, 4.0, 4.0)) if celltype == fcg.HEX8 else ((6, 2, 2), (6.0, 2.0, 2.0))


def _run_two_rank_solve(kinem, path, transport, solver="pcg", celltype=fcg.HEX8, world=2, stats=None):
    """The `world`-rank DistributedNewton of the clamped, tip-loaded box against the 1-rank
    StaticNewton (by DOF GID); returns the ranks' linear iteration counts (and appends each rank's
    fcg_amg_coupled_stats to `stats`)."""
    dev = _dev()
    newton = importlib.import_module("4c_amd.newton")
    iv, up = _solve_box(celltype)
    m = fcg.BoxMesh(celltype, iv, upper=up, jitter=0.1 if celltype == fcg.HEX8 else 0.02, seed=5)
    fext, dbc = _cantilever_loads(m, up[0])
    ev = fcg.Evaluator(m, kinematics=kinem, youngs=E, poisson=NU, device=0, path=path)
    ref = newton.StaticNewton(ev, fext, dbc, tol_res=1e-10, tol_inc=1e-11, lin_rtol=1e-12).solve()
    uref = dict(zip(m.row_gid.tolist(), ref.cpu().numpy().tolist()))
    ev.close()
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    qq = ctx.Queue()
    port = 29700 + os.getpid() % 1000
    procs = [ctx.Process(target=_worker_solve, args=(r, world, port, qq, kinem, path, transport, solver,
                                                     celltype)) for r in range(world)]
    for p in procs:
        p.start()
    res = [qq.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    got, iters = {}, []
    for rank, ok, out in sorted(res, key=lambda t: t[0]):
        assert ok is True, (rank, ok)
        got.update(out["u"])
        iters.append(out["iters"])
        if stats is not None:
            stats.append(out["stats"])
        if solver == "native":
            assert out["coupled_levels"] >= 1, out  # the coarse levels span both ranks
        elif solver == "native-uncoupled":
            assert out["coupled_levels"] == 0, out
    assert set(got) == set(uref)
    scale = max(abs(v) for v in uref.values())
    assert scale > 0
    worst = max(abs(got[g] - uref[g]) for g in uref)
    assert worst <= 1e-8 * scale, (worst, scale)
    assert dev is not None
    return iters


@pytest.mark.parametrize("solver", ["native", "native-bj"])
@pytest.mark.parametrize("celltype,kinem", [(fcg.HEX8, fcg.LINEAR), (fcg.HEX27, fcg.TOTLAG)])
def test_two_ranks_native_dfcg(celltype, kinem, solver):
    """fcg_dfcg_solve (the native distributed flexible CG: one import per SpMV, all-reduced inner
    products) with each rank's fcg_amg on its owned block ("native") or the nodal block Jacobi,
    inside the 2-rank Newton, host-staged transport callbacks on one GPU: the 1-rank solution."""
    iters = _run_two_rank_solve(kinem, fcg.PATH_AUTO, "staged", solver, celltype)
    if solver == "native":
        bj = _run_two_rank_solve(kinem, fcg.PATH_AUTO, "staged", "native-bj", celltype)
        assert sum(i or 0 for i in iters[0]) < sum(i or 0 for i in bj[0]), (iters, bj)
        # coarse levels coupled across the ranks (4C's MueLu hierarchy spans every rank,
        # 4C_linear_solver_preconditioner_muelu.cpp:97): the 2-rank solve needs at most 1.5x the
        # FCG iterations of the 1-rank AMG on the same problem; the rank-local subdomain AMG
        # (round 3) is kept as "native-uncoupled" for the comparison
        one = _one_rank_amg_iters(celltype, kinem)
        unc = _run_two_rank_solve(kinem, fcg.PATH_AUTO, "staged", "native-uncoupled", celltype)
        n1, n2, nu = sum(one), sum(i or 0 for i in iters[0]), sum(i or 0 for i in unc[0])
        print(f"FCG iterations: 1 rank {one}, 2 ranks coupled {iters[0]}, 2 ranks rank-local {unc[0]}")
        assert n2 <= 1.5 * n1, (one, iters, unc)
        assert n2 <= nu, (iters, unc)


@pytest.mark.parametrize("dist", ["0", "1"])
def test_two_ranks_native_dfcg_rccl(dist):
    """The coupled AMG path of fcg_dfcg_solve over the library's RCCL transport (fcg_transport_rccl
    names rank / nranks, so every RCCL solve with an AMG handle couples its coarse levels): one GPU
    per rank, the 1-rank solution, coupled levels >= 1 and the 1.5x iteration bound;
    dist "1": level 1 distributed, its exchanges through fcg_comm_exchange_device."""
    _dev()
    if torch.cuda.device_count() < 2:
        pytest.skip("RCCL transport needs two GPUs (RCCL refuses two ranks on one device)")
    st = []
    with _env(FCG_AMG_DIST=dist):
        iters = _run_two_rank_solve(fcg.LINEAR, fcg.PATH_AUTO, "rccl", "native", fcg.HEX8, stats=st)
    assert all(s_["distributed_levels"] == int(dist) for s_ in st), st
    one = _one_rank_amg_iters(fcg.HEX8, fcg.LINEAR)
    assert sum(i or 0 for i in iters[0]) <= 1.5 * sum(one), (one, iters)


def test_coupled_amg_setup_failure_on_one_rank_fails_every_rank():
    """A rank whose local AMG setup fails (injected on rank 1) must not leave rank 0 waiting in the
    coupled levels' collectives: fcg_amg_precond_setup all-reduces a go/no-go flag first, so both
    ranks' solves raise."""
    _dev()
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    qq = ctx.Queue()
    port = 29700 + (os.getpid() + 7) % 1000
    old = os.environ.get("FCG_AMG_INJECT_FAIL_RANK")
    os.environ["FCG_AMG_INJECT_FAIL_RANK"] = "1"
    try:
        procs = [ctx.Process(target=_worker_solve, args=(r, 2, port, qq, fcg.LINEAR, fcg.PATH_AUTO,
                                                         "staged", "native")) for r in range(2)]
        for p in procs:
            p.start()
    finally:
        if old is None:
            del os.environ["FCG_AMG_INJECT_FAIL_RANK"]
        else:
            os.environ["FCG_AMG_INJECT_FAIL_RANK"] = old
    try:
        res = sorted(qq.get(timeout=180) for _ in range(2))
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.terminate()
    assert [r for r, _, _ in res] == [0, 1]
    for rank, ok, _ in res:
        assert ok is not True, (rank, ok)
    assert "another rank" in res[0][1], res[0][1][-400:]
    assert "injected" in res[1][1], res[1][1][-400:]


@pytest.mark.parametrize("world,at", [(2, 0), (2, 3), (4, 1), (4, 6)])
def test_coupled_amg_failure_inside_the_build_fails_every_rank(world, at):
    """Rank 1 throws inside the coupled AMG build (FCG_AMG_INJECT_BUILD_FAIL="1:at": on reaching its
    at-th collective of the build, with level 1 distributed so the build's exchanges run) while the
    other ranks are inside the build's imports and exchanges.  The build runs over a transport
    whose collectives are preceded by a status all-reduce, so every rank's solve returns an error
    (rank 1 its own, the others "another rank") instead of leaving them waiting (gloo transport)."""
    _dev()
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    qq = ctx.Queue()
    port = 29700 + (os.getpid() + 11 + at) % 1000
    with _env(FCG_AMG_INJECT_BUILD_FAIL=f"1:{at}", FCG_AMG_DIST="1"):
        procs = [ctx.Process(target=_worker_solve, args=(r, world, port, qq, fcg.LINEAR, fcg.PATH_AUTO,
                                                         "staged", "native")) for r in range(world)]
        for p in procs:
            p.start()
    try:
        res = sorted(qq.get(timeout=180) for _ in range(world))
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.terminate()
    assert [r for r, _, _ in res] == list(range(world))
    for rank, ok, _ in res:
        assert ok is not True, (rank, ok)
        want = "injected" if rank == 1 else "another rank"
        assert want in res[rank][1], res[rank][1][-400:]


@pytest.mark.parametrize("world", [4, 8])
def test_many_ranks_coupled_amg_iterations(world):
    """The coupled coarse levels at 4 and 8 ranks (host-staged on one GPU, hex8 linear box): the
    solution by GID matches one rank, and the FCG iterations stay within 1.5x of the 1-rank AMG's
    (the rank-local AMG grows with the rank count)."""
    one = _one_rank_amg_iters(fcg.HEX8, fcg.LINEAR)
    iters = _run_two_rank_solve(fcg.LINEAR, fcg.PATH_AUTO, "staged", "native", fcg.HEX8, world=world)
    n1, nR = sum(one), sum(i or 0 for i in iters[0])
    print(f"FCG iterations: 1 rank {one}, {world} ranks coupled {iters[0]}")
    assert nR <= 1.5 * n1, (one, iters)


class _env:
    """Environment variables for the spawned ranks (they inherit os.environ at start)."""

    def __init__(self, **kv):
        self.kv, self.old = kv, {}

    def __enter__(self):
        for k, v in self.kv.items():
            self.old[k] = os.environ.get(k)
            os.environ[k] = v

    def __exit__(self, *exc):
        for k, v in self.old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.mark.parametrize("world", [2, 4, 8])
def test_distributed_level1_coupled_amg(world):
    """Level 1 of the coupled AMG distributed across the ranks (FCG_AMG_DIST=1: each rank owns the
    rows of its aggregates, the partial rows of the others' aggregates go to their owners through
    the transport's exchange, its own level-1 import plan; A_2 = T_1^T A_1 T_1 replicated): the
    1-rank solution by GID, the FCG iterations within 1.5x of one rank, and the stats -- the rank
    stores only its own level-1 rows, and the all-reduces carry level 2, not level 1."""
    one = _one_rank_amg_iters(fcg.HEX8, fcg.LINEAR)
    st_d, st_r = [], []
    with _env(FCG_AMG_DIST="1"):
        it_d = _run_two_rank_solve(fcg.LINEAR, fcg.PATH_AUTO, "staged", "native", fcg.HEX8, world=world,
                                   stats=st_d)
    with _env(FCG_AMG_DIST="0"):
        it_r = _run_two_rank_solve(fcg.LINEAR, fcg.PATH_AUTO, "staged", "native", fcg.HEX8, world=world,
                                   stats=st_r)
    n1, nd, nr = sum(one), sum(i or 0 for i in it_d[0]), sum(i or 0 for i in it_r[0])
    print(f"FCG iterations: 1 rank {one}, {world} ranks distributed level 1 {it_d[0]}, replicated {it_r[0]}")
    print("stats distributed", st_d, "replicated", st_r)
    assert nd <= 1.5 * n1, (one, it_d, it_r)
    glob = st_r[0]["level1_rows_global"]
    assert sum(s["level1_rows_here"] for s in st_d) == glob  # every level-1 row on exactly one rank
    for sd, sr in zip(st_d, st_r):
        assert sd["distributed_levels"] == 1 and sr["distributed_levels"] == 0
        assert sd["level1_rows_global"] == glob and sr["level1_rows_here"] == glob
        assert sd["exchange_doubles_apply"] > 0 and sr["exchange_doubles_apply"] == 0
        assert sr["allreduce_doubles_apply"] == 6 * glob
        assert sd["allreduce_doubles_apply"] < sr["allreduce_doubles_apply"]
        assert sd["allreduce_doubles_setup"] < sr["allreduce_doubles_setup"]
        assert sd["replicated_bytes"] < sr["replicated_bytes"]


def test_distributed_level1_weak_scaling_stats():
    """Weak scaling of the distributed level 1 (a box of 8 x 8 x 8 hex8 per rank along x, 2 and 4
    ranks): the level-1 rows and the exchange volume per rank stay put (within the boundary ranks'
    difference), while the replicated path's per-rank level-1 storage doubles with the ranks."""
    per = {}
    for world in (2, 4):
        st_d, st_r = [], []
        with _env(FCG_AMG_DIST="1", FCG_TEST_SOLVE_BOX=f"{8 * world},8,8"):
            _run_two_rank_solve(fcg.LINEAR, fcg.PATH_AUTO, "staged", "native", fcg.HEX8, world=world, stats=st_d)
        with _env(FCG_AMG_DIST="0", FCG_TEST_SOLVE_BOX=f"{8 * world},8,8"):
            _run_two_rank_solve(fcg.LINEAR, fcg.PATH_AUTO, "staged", "native", fcg.HEX8, world=world, stats=st_r)
        per[world] = (max(s["level1_rows_here"] for s in st_d), max(s["exchange_doubles_apply"] for s in st_d),
                      max(s["level1_rows_here"] for s in st_r))
        print(world, "distributed", st_d, "replicated", st_r)
    (r2, x2, g2), (r4, x4, g4) = per[2], per[4]
    assert r4 <= 1.25 * r2 and x4 <= 2.25 * x2, per  # interior ranks exchange on two faces
    assert g4 >= 1.8 * g2, per


@pytest.mark.parametrize("world", [2, 4])
def test_distributed_deeper_levels_coupled_amg(world):
    """Levels 1..k of the coupled AMG distributed (FCG_AMG_DIST_MIN=0: every coarser level that
    still shrinks is distributed too, FCG_AMG_DIST_LEVELS=3 caps them; each level a Dist of its own,
    built from the partial rows of the level above): the 1-rank solution by GID, the FCG iterations
    within 1.5x of one rank, and the stats against level 1 alone -- more distributed levels, a
    smaller replicated level, fewer doubles all-reduced per application."""
    box = "32,12,12"
    with _env(FCG_TEST_SOLVE_BOX=box):
        one = _one_rank_amg_iters(fcg.HEX8, fcg.LINEAR)
    st1, stk = [], []
    with _env(FCG_AMG_DIST="1", FCG_AMG_DIST_LEVELS="1", FCG_TEST_SOLVE_BOX=box):
        it1 = _run_two_rank_solve(fcg.LINEAR, fcg.PATH_AUTO, "staged", "native", fcg.HEX8, world=world, stats=st1)
    with _env(FCG_AMG_DIST="1", FCG_AMG_DIST_MIN="0", FCG_AMG_DIST_LEVELS="3", FCG_TEST_SOLVE_BOX=box):
        itk = _run_two_rank_solve(fcg.LINEAR, fcg.PATH_AUTO, "staged", "native", fcg.HEX8, world=world, stats=stk)
    n1, na, nk = sum(one), sum(i or 0 for i in it1[0]), sum(i or 0 for i in itk[0])
    print(f"FCG iterations: 1 rank {one}, {world} ranks level 1 distributed {it1[0]}, levels 1..k {itk[0]}")
    print("stats level 1", st1, "levels 1..k", stk)
    assert na <= 1.5 * n1 and nk <= 1.5 * n1, (one, it1, itk)
    for a, b in zip(st1, stk):
        assert a["distributed_levels"] == 1 and b["distributed_levels"] >= 2, (a, b)
        assert a["level1_rows_here"] == b["level1_rows_here"]
        assert b["replicated_rows"] < a["replicated_rows"]
        assert b["replicated_bytes"] < a["replicated_bytes"]
        assert b["allreduce_doubles_apply"] == 6 * b["replicated_rows"]
        assert b["allreduce_doubles_apply"] < a["allreduce_doubles_apply"]
    assert len({s["distributed_levels"] for s in stk}) == 1  # every rank decided alike


def test_distributed_levels_weak_scaling_replicated_bounded():
    """Weak scaling with the replication threshold (a box of 12 x 12 x 12 hex8 per rank along x on
    2, 4 and 8 ranks, FCG_AMG_DIST_MIN=72 DOFs): the levels past the threshold are distributed, so
    the replicated level stays under it at every rank count (or at one aggregate per rank, the floor
    of a rank-local aggregation), while with level 1 alone distributed the replicated level grows
    with the ranks; the FCG iterations stay within 1.5x of one rank."""
    thr = 72
    per = {}
    for world in (2, 4, 8):
        box = f"{12 * world},12,12"
        with _env(FCG_TEST_SOLVE_BOX=box):
            one = _one_rank_amg_iters(fcg.HEX8, fcg.LINEAR)
        st_k, st_1 = [], []
        with _env(FCG_AMG_DIST="1", FCG_AMG_DIST_MIN=str(thr), FCG_TEST_SOLVE_BOX=box):
            itk = _run_two_rank_solve(fcg.LINEAR, fcg.PATH_AUTO, "staged", "native", fcg.HEX8, world=world,
                                      stats=st_k)
        with _env(FCG_AMG_DIST="1", FCG_AMG_DIST_LEVELS="1", FCG_TEST_SOLVE_BOX=box):
            _run_two_rank_solve(fcg.LINEAR, fcg.PATH_AUTO, "staged", "native", fcg.HEX8, world=world, stats=st_1)
        n1, nk = sum(one), sum(i or 0 for i in itk[0])
        print(world, "iterations 1 rank", one, "distributed", itk[0], "stats", st_k, "level 1 only", st_1)
        assert nk <= 1.5 * n1, (world, one, itk)
        per[world] = (st_k[0]["replicated_rows"], st_k[0]["distributed_levels"], st_1[0]["replicated_rows"],
                      max(s["replicated_bytes"] for s in st_k), max(s["replicated_bytes"] for s in st_1))
    print(per)
    for world, (rk, lk, r1, bk, b1) in per.items():
        assert 6 * rk <= max(thr, 6 * world), per  # under the threshold (or one aggregate per rank)
        assert rk <= r1 and bk <= b1, per
    assert per[8][1] >= 2 and per[8][0] < per[8][2], per  # 8 ranks: level 2 distributed too
    assert per[8][2] >= 3 * per[2][2], per  # level 1 alone: the replicated level grows with the ranks


def _one_rank_amg_iters(celltype, kinem):
    """The same Newton on one rank with the native AMG (fcg_amg_iterate): FCG iterations per step."""
    _dev()
    newton = importlib.import_module("4c_amd.newton")
    amg_mod = importlib.import_module("4c_amd.amg")
    iv, up = _solve_box(celltype)
    m = fcg.BoxMesh(celltype, iv, upper=up, jitter=0.1 if celltype == fcg.HEX8 else 0.02, seed=5)
    fext, dbc = _cantilever_loads(m, up[0])
    ev = fcg.Evaluator(m, kinematics=kinem, youngs=E, poisson=NU, device=0)
    amg = amg_mod.NativeAMG(m, ev, dbc)
    nt = newton.StaticNewton(ev, fext, dbc, tol_res=1e-10, tol_inc=1e-11, lin_rtol=1e-12,
                             linear_solver=amg)
    nt.solve()
    its = [r.get("lin_iter") or 0 for r in nt.history]
    amg.close()
    ev.close()
    return its


@pytest.mark.parametrize("transport", ["staged", "rccl"])
@pytest.mark.parametrize("kinem,path", [(fcg.LINEAR, fcg.PATH_AUTO), (fcg.TOTLAG, fcg.PATH_GENERAL)])
def test_two_ranks_distributed_newton_pcg(kinem, path, transport):
    """dsolve.DistributedNewton on 2 ranks (halo import before every SpMV, global dots) converges
    to the 1-rank StaticNewton solution of the same clamped, tip-loaded box (by DOF GID).
    transport "staged": both ranks on GPU 0, host-staged gloo; "rccl": one GPU per rank with the
    RCCL halo and all-reduce inside the solver loop (needs two GPUs; RCCL refuses two ranks on one)."""
    dev = _dev()
    if transport == "rccl" and torch.cuda.device_count() < 2:
        pytest.skip("RCCL transport needs two GPUs (RCCL refuses two ranks on one device)")
    newton = importlib.import_module("4c_amd.newton")
    iv, up = (8, 4, 4), (8.0, 4.0, 4.0)
    m = fcg.BoxMesh(fcg.HEX8, iv, upper=up, jitter=0.1, seed=5)
    fext, dbc = _cantilever_loads(m, up[0])
    ev = fcg.Evaluator(m, kinematics=kinem, youngs=E, poisson=NU, device=0, path=path)
    # tolerances above the f_int rounding floor (TotLag stalls near 1e-12 absolute here)
    ref = newton.StaticNewton(ev, fext, dbc, tol_res=1e-10, tol_inc=1e-11, lin_rtol=1e-12).solve()
    uref = dict(zip(m.row_gid.tolist(), ref.cpu().numpy().tolist()))
    ev.close()
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    qq = ctx.Queue()
    port = 29700 + os.getpid() % 1000
    procs = [ctx.Process(target=_worker_solve, args=(r, 2, port, qq, kinem, path, transport))
             for r in range(2)]
    for p in procs:
        p.start()
    res = [qq.get(timeout=240) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
    got = {}
    for rank, ok, out in res:
        assert ok is True, (rank, ok)
        got.update(out["u"])
    assert set(got) == set(uref)
    scale = max(abs(v) for v in uref.values())
    assert scale > 0
    worst = max(abs(got[g] - uref[g]) for g in uref)
    assert worst <= 1e-8 * scale, (worst, scale)
    assert dev is not None


def test_native_amg_refuses_to_solve_on_a_rank_of_a_partition():
    """A NativeAMG built on a rank of a 2-rank partition covers the owned block only: solving with
    it alone would answer the block-diagonal local system.  fcg_amg_iterate / fcg_amg_solve refuse
    (FCG_ERR_ARG, pointing at fcg_dfcg_solve), and so does NativeAMG.solve; setup and apply -- the
    preconditioner role inside fcg_dfcg_solve -- still work."""
    dev = _dev()
    amg_mod = importlib.import_module("4c_amd.amg")
    import ctypes
    iv, up = _solve_box(fcg.HEX8)
    m = fcg.BoxMesh(fcg.HEX8, iv, upper=up, jitter=0.1, seed=5, rank=0, nranks=2)
    assert m.n_cols > m.n_rows
    ev = fcg.Evaluator(m, kinematics=fcg.LINEAR, youngs=E, poisson=NU, device=0)
    fext, dbc = _cantilever_loads(m, up[0])
    amg = amg_mod.NativeAMG(m, ev, dbc)
    assert amg.local
    K = torch.zeros(int(ev.info.nnz), dtype=torch.float64, device=dev)
    f = torch.zeros(m.n_rows, dtype=torch.float64, device=dev)
    u = torch.zeros(m.n_cols, dtype=torch.float64, device=dev)
    ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, u, f, K)
    # rank 0 holds no tip load: a random right-hand side, zero on the Dirichlet rows
    rhs = np.random.default_rng(1).standard_normal(m.n_rows)
    rhs[dbc] = 0.0
    b = torch.from_numpy(rhs).to(dev)
    x = torch.zeros_like(b)
    with pytest.raises(fcg.FcgError) as ei:
        amg.solve(K, b, x, 1e-8)
    assert ei.value.code == 3 and "fcg_dfcg_solve" in str(ei.value)
    L = fcg.lib()
    vp = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    it, rel = ctypes.c_int(0), ctypes.c_double(0.0)
    s = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    rc = L.fcg_amg_solve(amg._h, vp(K), vp(b), vp(x), 1e-8, 100, ctypes.byref(it), ctypes.byref(rel), s)
    assert rc == 3 and b"fcg_dfcg_solve" in L.fcg_amg_last_error(amg._h)
    amg.setup(K)
    rc = L.fcg_amg_iterate(amg._h, vp(K), vp(b), vp(x), 1e-8, 100, ctypes.byref(it), ctypes.byref(rel), s)
    assert rc == 3 and it.value == 0
    z = torch.zeros_like(b)
    assert L.fcg_amg_apply(amg._h, vp(K), vp(b), vp(z), s) == 0
    torch.cuda.synchronize()
    assert torch.isfinite(z).all() and float(z.abs().max()) > 0
    amg.close()
    ev.close()
