"""Two-field TSI tangent on one GPU (BASELINE config 5 per-GPU share): one assembly of
k_SS + f_S (structured sweep) and k_ST, k_TS, k_TT, f_T, f_S(T) (TSI kernels), hex8 linear,
ThermoStVenantKirchhoff + Fourier -- as two calls (sweep + TSI kernels) and as the fused sweep
(fcg_tsi_evaluate_fused).  Prints one JSON line.
usage: tsi_bench.py [--n N] [--reps R]"""
import argparse
import importlib
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
fcg = importlib.import_module("4c_amd").fcg
ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=126)
ap.add_argument("--reps", type=int, default=10)
a = ap.parse_args()
E, NU, ALPHA, T0, COND, DT = 210.0, 0.3, 1.2e-5, 293.0, 52.0, 0.5
dev = torch.device("cuda:0")
t0 = time.perf_counter()
m = fcg.BoxMesh(fcg.HEX8, (a.n, a.n, a.n), jitter=0.1)
ev = fcg.Evaluator(m, kinematics=fcg.LINEAR, youngs=E, poisson=NU, path=fcg.PATH_STRUCTURED)
tev = fcg.TsiEvaluator(m, E, NU, ALPHA, T0, COND)
g = tev.graph
t_setup = time.perf_counter() - t0
X = m.node_x
T = torch.from_numpy(T0 + 50.0 * np.sin(2 * np.pi * X[:, 0]) * np.cos(np.pi * X[:, 1])).to(dev)
u = torch.from_numpy(m.u_col(1e-3)).to(dev)
v = torch.from_numpy(m.u_col(1e-2)).to(dev)
f64 = dict(dtype=torch.float64, device=dev)
fs, Kss = torch.zeros(m.n_rows, **f64), torch.zeros(m.nnz, **f64)
o = {k: torch.zeros(n, **f64) for k, n in (("Kst", g.nnz_st), ("Kts", g.nnz_ts), ("Ktt", g.nnz_tt),
                                           ("fT", g.n_rows_t))}
s = torch.cuda.current_stream(dev)


def step():
    ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, u, fs, Kss, stream=s)
    e1.record(s)
    tev.evaluate_device(fcg.TSI_ALL, fcg.OVERWRITE, v, T, 1.0, 1.0 / DT, fs=fs, stream=s, **o)


e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
for _ in range(2):
    step()
ms_s, ms_t = [], []
for _ in range(a.reps):
    e0.record(s)
    step()
    e2.record(s)
    torch.cuda.synchronize()
    ms_s.append(e0.elapsed_time(e1))
    ms_t.append(e1.elapsed_time(e2))
ms_s, ms_t = float(np.median(ms_s)), float(np.median(ms_t))
fused = dict(fs=fs, Kss=Kss, **o)
for _ in range(2):
    tev.evaluate_fused(ev, fcg.OVERWRITE, u, v, T, 1.0, 1.0 / DT, stream=s, **fused)
ms_f = []
for _ in range(a.reps):
    e0.record(s)
    tev.evaluate_fused(ev, fcg.OVERWRITE, u, v, T, 1.0, 1.0 / DT, stream=s, **fused)
    e2.record(s)
    torch.cuda.synchronize()
    ms_f.append(e0.elapsed_time(e2))
ms_f = float(np.median(ms_f))
# algorithmic HBM bytes of the fused pass: the four matrices and two residuals written once,
# coordinates / u / v / T read once per node
byt = 8 * (m.nnz + g.nnz_st + g.nnz_ts + g.nnz_tt + m.n_rows + g.n_rows_t) + 8 * 10 * m.n_node
print(json.dumps({"config": f"tsi-hex8-linear-{a.n}^3", "elements": m.n_ele,
                  "nnz_ss": m.nnz, "nnz_st": g.nnz_st, "nnz_ts": g.nnz_ts, "nnz_tt": g.nnz_tt,
                  "ms_structure": ms_s, "ms_tsi_blocks": ms_t, "ms_two_field_tangent": ms_s + ms_t,
                  "elem_per_s": m.n_ele / ((ms_s + ms_t) * 1e-3), "ms_fused": ms_f,
                  "fused_elem_per_s": m.n_ele / (ms_f * 1e-3),
                  "fused_hbm_gbs": byt / (ms_f * 1e-3) / 1e9, "setup_s": t_setup}))
