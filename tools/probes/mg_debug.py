"""Multigrid diagnostics: per level, the operator against torch's CSR product, the Rayleigh
quotient of random vectors and the Lanczos eigenvalue estimates (development aid)."""
import importlib, os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
fcg = importlib.import_module("4c_amd").fcg
mgm = importlib.import_module("4c_amd.multigrid")
ct = fcg.HEX27 if sys.argv[1] == "hex27" else fcg.HEX8
n = int(sys.argv[2])
mesh = fcg.BoxMesh(ct, (n, n, n))
ev = fcg.Evaluator(mesh, kinematics=fcg.LINEAR, youngs=210.0, poisson=0.3)
dev = torch.device("cuda:0")
f64 = dict(dtype=torch.float64, device=dev)
K = torch.zeros(mesh.nnz, **f64)
ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, torch.zeros(mesh.n_cols, **f64), torch.zeros(mesh.n_rows, **f64), K)
clamp = lambda m: np.isclose(m.node_x[:, 0], 0.0)
nodes = np.nonzero(clamp(mesh))[0]
dbc = np.sort((mesh.node_dof_row[nodes][:, None] + np.arange(3)).ravel()).astype(np.int32)
ev.dirichlet_apply(torch.as_tensor(dbc, device=dev), K)
mg = mgm.Multigrid(mesh, ev, clamp, 210.0, 0.3, min_intervals=2)
mg.levels[0].K = K
mg.levels[0].setup_diag()
print("col==row map:", np.array_equal(mesh.node_dof_col, mesh.node_dof_row))
for l, lvl in enumerate(mg.levels):
    m = lvl.mesh
    A = torch.sparse_csr_tensor(torch.from_numpy(m.rowptr).to(dev), torch.from_numpy(m.col_lid.astype(np.int64)).to(dev), lvl.K, size=(m.n_rows, m.n_cols))
    x = torch.randn(m.n_rows, **f64) * lvl.mask
    y = torch.empty_like(x)
    lvl.spmv(x, y)
    y2 = A @ x
    z = torch.empty_like(x)
    lvl.apply_dinv(x, z)
    print(l, "n", m.n_rows, "spmv err", float((y - y2).abs().max() / y2.abs().max()), "xAx", float(x @ y),
          "xDinvx", float(x @ z), "col==row", np.array_equal(m.node_dof_col, m.node_dof_row), flush=True)
    lvl.estimate_lmax()
    print("   lanczos lmax", lvl.lmax, flush=True)
