"""Run one configuration's evaluate a few times (for rocprofv3 counter passes)."""
import argparse
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
fcg = importlib.import_module("4c_amd").fcg

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=100)
ap.add_argument("--celltype", default="hex8")
ap.add_argument("--kinem", default="linear")
ap.add_argument("--path", default="auto")
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--seed", type=int, default=20251015, help="jitter seed (bench.py's mesh)")
ap.add_argument("--renumber", action="store_true", help="random node/element numbering (input-file mesh)")
ap.add_argument("--tsi", action="store_true", help="the fused TSI two-field tangent (config 5)")
a = ap.parse_args()
ct = fcg.HEX8 if a.celltype == "hex8" else fcg.HEX27
kin = fcg.LINEAR if a.kinem == "linear" else fcg.TOTLAG
path = {"auto": fcg.PATH_AUTO, "general": fcg.PATH_GENERAL, "structured": fcg.PATH_STRUCTURED,
        "gather": fcg.PATH_GATHER, "colored": fcg.PATH_COLORED}[a.path]
m = fcg.BoxMesh(ct, (a.n, a.n, a.n), jitter=0.1 if ct == fcg.HEX8 else 0.02, seed=a.seed)
if a.renumber:
    box = m
    m = fcg.Discretization.renumbered(box, seed=1)
    m.u_col = lambda amp: np.random.default_rng(3).standard_normal(m.n_cols) * amp
ev = fcg.Evaluator(m, kinematics=kin, path=path)
dev = torch.device("cuda:0")
if a.tsi:
    E, NU, ALPHA, T0, COND, DT = 210.0, 0.3, 1.2e-5, 293.0, 52.0, 0.5
    tev = fcg.TsiEvaluator(m, E, NU, ALPHA, T0, COND)
    g = tev.graph
    X = m.node_x
    T = torch.from_numpy(T0 + 50.0 * np.sin(2 * np.pi * X[:, 0]) * np.cos(np.pi * X[:, 1])).to(dev)
    u = torch.from_numpy(m.u_col(1e-3)).to(dev)
    v = torch.from_numpy(m.u_col(1e-2)).to(dev)
    f64 = dict(dtype=torch.float64, device=dev)
    o = dict(fs=torch.zeros(m.n_rows, **f64), Kss=torch.zeros(m.nnz, **f64),
             Kst=torch.zeros(g.nnz_st, **f64), Kts=torch.zeros(g.nnz_ts, **f64),
             Ktt=torch.zeros(g.nnz_tt, **f64), fT=torch.zeros(g.n_rows_t, **f64))
    for _ in range(a.reps):
        tev.evaluate_fused(ev, fcg.OVERWRITE, u, v, T, 1.0, 1.0 / DT, **o)
    torch.cuda.synchronize()
    print("tsi fused ok")
    sys.exit(0)
u = torch.from_numpy(m.u_col(1e-3 if kin == fcg.LINEAR else 5e-2)).to(dev)
f = torch.zeros(m.n_rows, dtype=torch.float64, device=dev)
K = torch.zeros(m.nnz, dtype=torch.float64, device=dev)
for _ in range(a.reps):
    ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, u, f, K)
torch.cuda.synchronize()
print("path", ev.info.path, "ok")
