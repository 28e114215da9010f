"""World-size-2 (and 4) gloo tests of the multi-rank host path on CPU: the displacement import
(set_state) moves exactly the ghost DOFs and reproduces the global column vector, and the
residual norm all-reduce equals the global norm."""

import importlib
import os
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(rank, world, port, q):
    try:
        sys.path.insert(0, ROOT)
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        pkg = importlib.import_module("4c_amd")
        fcg = pkg.fcg
        halo = importlib.import_module("4c_amd.halo")
        iv = (6, 5, 4)
        glob = fcg.BoxMesh(fcg.HEX8, iv)
        ug = glob.u_col(1e-3)
        gmap = {int(g): i for i, g in enumerate(glob.col_gid)}
        m = fcg.BoxMesh(fcg.HEX8, iv, rank=rank, nranks=world)
        owner = halo.col_owner_of(m)
        imp = halo.HaloImport(m.row_gid, m.col_gid, owner, rank, world, torch.device("cpu"))
        assert imp.contiguous  # BoxMesh column maps: owned prefix + ghosts by (owner, gid)
        u_row = torch.tensor([ug[gmap[int(g)]] for g in m.row_gid], dtype=torch.float64)
        u_col = torch.full((m.n_cols,), float("nan"), dtype=torch.float64)
        imp(u_row, u_col)
        expect = np.array([ug[gmap[int(g)]] for g in m.col_gid])
        ok = np.array_equal(u_col.numpy(), expect)
        # residual norm over ranks == global norm of the owned pieces
        nrm = halo.residual_norm(u_row).item()
        q.put((rank, ok, imp.n_ghost, nrm, float(np.linalg.norm(ug))))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, repr(e), -1, 0.0, 0.0))


@pytest.mark.parametrize("world", [2, 4])
def test_halo_import_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + world * 7 + os.getpid() % 1000
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for rank, ok, nghost, nrm, gnrm in res:
        assert ok is True, (rank, ok)
        assert nghost > 0
        assert abs(nrm - gnrm) <= 1e-12 * gnrm
