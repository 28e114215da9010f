"""Operator (fcg_spmv, y = K x by node rows) bandwidth on one GPU: K assembled by fcg_evaluate_device
on a box mesh, then R timed applications (hipEvents around the loop).  Bytes per apply: the K
values, one column index per 3x3 block, x (once) and y.
usage: spmv_bench.py [--celltype hex27] [--n 50] [--reps 50]"""
import argparse
import importlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
fcg = importlib.import_module("4c_amd").fcg
ap = argparse.ArgumentParser()
ap.add_argument("--celltype", default="hex27")
ap.add_argument("--n", type=int, default=50)
ap.add_argument("--reps", type=int, default=50)
a = ap.parse_args()
ct = fcg.HEX8 if a.celltype == "hex8" else fcg.HEX27
m = fcg.BoxMesh(ct, (a.n, a.n, a.n), jitter=0.02)
ev = fcg.Evaluator(m, kinematics=fcg.LINEAR)
dev = torch.device("cuda:0")
u = torch.from_numpy(m.u_col(1e-3)).to(dev)
f = torch.zeros(m.n_rows, dtype=torch.float64, device=dev)
K = torch.zeros(m.nnz, dtype=torch.float64, device=dev)
ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, u, f, K)
y = torch.zeros(m.n_rows, dtype=torch.float64, device=dev)
s = torch.cuda.current_stream(dev)
for _ in range(3):
    ev.spmv(K, u, y, stream=s)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(s)
for _ in range(a.reps):
    ev.spmv(K, u, y, stream=s)
e1.record(s)
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / a.reps
err = (torch.linalg.norm(y - f) / torch.linalg.norm(f)).item()  # K u = f_int (linear kinematics)
byt = 8 * m.nnz + 4 * (m.nnz // 9) + 8 * (m.n_cols + m.n_rows)
print(json.dumps({"config": f"{a.celltype}-{a.n}^3", "nnz": m.nnz, "ms_spmv": ms,
                  "gb_per_apply": byt / 1e9, "gbs": byt / (ms * 1e-3) / 1e9, "Ku_vs_f": err}))
