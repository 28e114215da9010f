"""BASELINE config 4 at its stated size: 8M hex8 (200^3) element-partitioned over 8 ranks.

The 8 ranks run in turn on the one GPU of the test box (RCCL refuses two ranks on one device; the
driver's 8-GPU node runs them concurrently in bench.py).  Everything a rank does on its own GPU runs
here through the library:

* the partition: 4C's GridGenerator split of the 200^3 box into 2 x 2 x 2 sub-boxes
  (4C_io_gridgenerator.cpp:85-153) with one layer of ghost elements
  (4C_fem_discretization_partition.cpp:510-543) -- fcg.BoxMesh(..., rank=r, nranks=8);
* set_state (4C_fem_discretization.cpp:540-550): every rank's import plan built by the library's
  fcg_import_plan_build, collectively over the 8 ranks (ranks as threads of this process,
  halo.run_ranks), the owned displacements packed on the device by fcg_halo_pack, the bytes moved
  host-side (what RCCL's grouped send / recv does on the node), scattered by fcg_halo_unpack;
* option A (the reference's semantics): each rank's evaluate of its column elements writes its
  owned rows only (4C_linalg_sparsematrix.cpp:474) -- compared with the oracle's rows of the same
  rank, K and f_int by (row GID, column GID) at 1e-12 / 1e-10;
* option B (north_star's shared-DOF all-reduce): the strict element partition, each rank's partial
  f_int packed by fcg_shared_pack, summed over the ranks (the ncclAllReduce of the interface
  buffer) and unpacked by fcg_shared_unpack -- compared with the oracle's strict partials reduced
  the same way and with option A's owned rows by DOF GID.
"""

import importlib

import numpy as np
import pytest

from parity_util import oracle_evaluate, rel_err

torch = pytest.importorskip("torch")
fcg = importlib.import_module("4c_amd").fcg
halo = importlib.import_module("4c_amd.halo")

pytestmark = pytest.mark.gpu

E, NU = 210.0, 0.3
N, WORLD, AMP = 200, 8, 1e-3


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


@pytest.fixture(scope="module")
def split():
    """The 8 ghosted ranks of the 200^3 box, their import plans (one collective build) and what each
    rank's fcg_halo_pack sends; plus the owned f_int rows by GID as the option-A test finds them."""
    dev = _dev()
    meshes = [fcg.BoxMesh(fcg.HEX8, (N, N, N), rank=r, nranks=WORLD) for r in range(WORLD)]
    assert sum(m.n_ele_row for m in meshes) == meshes[0].n_ele_global == N ** 3
    plans = halo.run_ranks(WORLD, lambda r, x: halo.ImportPlan(
        r, WORLD, meshes[r].row_gid, meshes[r].col_gid, halo.col_owner_of(meshes[r]), x))
    sends = []
    for m, plan in zip(meshes, plans):
        # Epetra column layout: the owned DOFs first, in row order
        assert plan.n_same == m.n_rows and plan.n_permute == 0
        h = halo.Halo(plan, 0)
        u_row = _t(m.u_col(AMP)[:m.n_rows], dev)
        u_col = torch.full((m.n_cols,), float("nan"), dtype=torch.float64, device=dev)
        send = torch.empty(max(1, h.n_send), dtype=torch.float64, device=dev)
        h.pack(u_row, u_col, send)
        torch.cuda.synchronize()
        sends.append(send[:h.n_send].cpu().numpy())
        h.close()
    return {"meshes": meshes, "plans": plans, "sends": sends, "f_by_gid": {}}


@pytest.mark.parametrize("ranks", [(0, 1), (2, 3), (4, 5), (6, 7)])
def test_config4_eight_rank_split_full_size(split, ranks):
    dev = _dev()
    meshes, plans, sends = split["meshes"], split["plans"], split["sends"]
    for r in ranks:
        m, plan = meshes[r], plans[r]
        # what rank r receives: peer p's segment for r follows p's segments for the ranks before r
        recv = np.concatenate([sends[p][int(plans[p].send_counts[:r].sum()):
                                        int(plans[p].send_counts[:r + 1].sum())] for p in range(WORLD)])
        assert len(recv) == int(plan.recv_counts.sum()) > 0
        h = halo.Halo(plan, 0)
        expect = m.u_col(AMP)
        u_col = torch.full((m.n_cols,), float("nan"), dtype=torch.float64, device=dev)
        send = torch.empty(max(1, h.n_send), dtype=torch.float64, device=dev)
        h.pack(_t(expect[:m.n_rows], dev), u_col, send)
        h.unpack(_t(recv, dev), u_col)
        torch.cuda.synchronize()
        h.close()
        u_host = u_col.cpu().numpy()
        assert np.array_equal(u_host, expect), r  # set_state: bit-exact column vector
        ev = fcg.Evaluator(m, kinematics=fcg.LINEAR, youngs=E, poisson=NU, device=0)
        assert ev.info.path == fcg.PATH_STRUCTURED  # the bench's fused sweep on every rank
        K = torch.full((m.nnz,), float("nan"), dtype=torch.float64, device=dev)
        f = torch.zeros(m.n_rows, dtype=torch.float64, device=dev)
        ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, u_col, f, K)
        torch.cuda.synchronize()
        ev.close()
        Kg, fg = K.cpu().numpy(), f.cpu().numpy()
        del K, f, u_col, send
        # the oracle on the same rank: its column elements, its owned rows, its CSR (row GID,
        # column GID through the rank's maps)
        err, _, Kr, fr = oracle_evaluate(m, fcg.LINEAR, E, NU, u_host, nworkers=16)
        assert err == 0
        assert np.all(np.isfinite(Kg)), r
        assert rel_err(fg, fr) <= 1e-10, (r, rel_err(fg, fr))
        assert rel_err(Kg, Kr) <= 1e-12, (r, rel_err(Kg, Kr))
        assert np.abs(Kg - Kr).max() <= 1e-12 * np.abs(Kr).max(), r
        split["f_by_gid"][r] = (m.row_gid.astype(np.int64), fg)
        del Kg, Kr


def test_config4_strict_partition_shared_dof_allreduce(split):
    """Option B at config 4's size: 8 strict ranks (row elements only), partial f_int on the GPU,
    the interface buffer summed over the ranks, owned rows = the oracle's reduced strict partials
    and = option A's owned rows (by GID)."""
    dev = _dev()
    strict = [fcg.BoxMesh(fcg.HEX8, (N, N, N), rank=r, nranks=WORLD, strict=True) for r in range(WORLD)]
    assert sum(m.n_ele for m in strict) == N ** 3  # no ghost elements
    sps = halo.run_ranks(WORLD, lambda r, x: halo.SharedPlan.of_mesh(strict[r], x))
    n_global = sps[0].n_global
    assert all(p.n_global == n_global for p in sps) and n_global > 0
    total_gpu, total_orc = np.zeros(n_global), np.zeros(n_global)
    keep = []
    for r, m in enumerate(strict):
        u = m.u_col(AMP)
        ev = fcg.Evaluator(m, kinematics=fcg.LINEAR, youngs=E, poisson=NU, device=0)
        f = torch.zeros(m.n_rows, dtype=torch.float64, device=dev)
        ev.evaluate_device(fcg.CALC_INTERNALFORCE, fcg.OVERWRITE, _t(u, dev), f, None)
        sh = halo.Shared(sps[r], 0)
        buf = torch.zeros(n_global, dtype=torch.float64, device=dev)
        sh.pack(f, buf)
        torch.cuda.synchronize()
        ev.close()
        total_gpu += buf.cpu().numpy()
        err, _, _, fo = oracle_evaluate(m, fcg.LINEAR, E, NU, u, want_k=False, nworkers=16)
        assert err == 0
        total_orc += sps[r].pack_host(fo)
        keep.append((f, sh, fo))
    assert rel_err(total_gpu, total_orc) <= 1e-10
    tot = _t(total_gpu, dev)
    for r, m in enumerate(strict):
        f, sh, fo = keep[r]
        sh.unpack(tot, f)
        torch.cuda.synchronize()
        own = f.cpu().numpy()[:m.n_owned_rows]
        sps[r].unpack_host(total_orc, fo)
        assert rel_err(own, fo[:m.n_owned_rows]) <= 1e-10, r
        if r in split["f_by_gid"]:  # option A's rows of the same DOFs (checked against the oracle)
            gid_a, fa = split["f_by_gid"][r]
            assert np.array_equal(gid_a, m.row_gid[:m.n_owned_rows].astype(np.int64))
            assert rel_err(own, fa) <= 1e-10, r
        sh.close()
