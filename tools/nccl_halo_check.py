"""Rehearsal of the RCCL halo import (HaloImport's contiguous path: owned copy + all_to_all_single
straight into the column vector's tail) with WORLD_SIZE ranks on the visible GPU(s); every rank
checks its column vector against the analytic field.  Launch with torch.distributed.run."""
import importlib, os, sys
import numpy as np
import torch
import torch.distributed as dist
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
fcg = importlib.import_module("4c_amd").fcg
halo = importlib.import_module("4c_amd.halo")
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count())
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)
m = fcg.BoxMesh(fcg.HEX8, (12 * world, 12, 12), rank=rank, nranks=world)
ref = m.u_col(1e-3)
row_lid = {int(g): i for i, g in enumerate(m.col_gid)}
u_row = torch.from_numpy(ref[[row_lid[int(g)] for g in m.row_gid]]).to(dev)
imp = halo.HaloImport(m.row_gid, m.col_gid, halo.col_owner_of(m), rank, world, dev)
u_col = torch.zeros(m.n_cols, dtype=torch.float64, device=dev)
imp(u_row, u_col)
torch.cuda.synchronize()
err = float(np.abs(u_col.cpu().numpy() - ref).max())
f = torch.ones(m.n_rows, dtype=torch.float64, device=dev)
nrm = float(halo.residual_norm(f))
print(f"rank {rank}: contiguous={imp.contiguous} ghosts={imp.n_ghost} max err {err:.1e} "
      f"|1|^2 over ranks {nrm ** 2:.1f}", flush=True)
assert err == 0.0
dist.barrier()
dist.destroy_process_group()
