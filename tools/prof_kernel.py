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
u = torch.from_numpy(m.u_col(1e-3 if kin == fcg.LINEAR else 5e-2)).to(dev)
f = torch.zeros(m.n_rows, dtype=torch.float64, device=dev)
K = torch.zeros(m.nnz, dtype=torch.float64, device=dev)
for _ in range(a.reps):
    ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, u, f, K)
torch.cuda.synchronize()
print("path", ev.info.path, "ok")
