"""Where the bench step's time goes beyond the kernel: evaluate alone (queued back to back), plus
the residual norm (one host round trip per step), plus the error check.  Prints ms per step."""
import importlib
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
fcg = importlib.import_module("4c_amd").fcg  # FCG_LIB selects an A/B build
halo = importlib.import_module("4c_amd.halo")
m = fcg.BoxMesh(fcg.HEX8, (100, 100, 100), jitter=0.1, seed=20251015)
ev = fcg.Evaluator(m, kinematics=fcg.LINEAR, youngs=210.0, poisson=0.3)
dev = torch.device("cuda:0")
u = torch.from_numpy(m.u_col(1e-3)).to(dev)
f = torch.zeros(m.n_rows, dtype=torch.float64, device=dev)
K = torch.zeros(m.nnz, dtype=torch.float64, device=dev)
s = torch.cuda.current_stream(dev)
ev.set_async(True)
fcg.measure_peaks(0)


def run(name, body, n=50):
    for _ in range(10):
        body()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        body()
    torch.cuda.synchronize()
    print(f"{name:40s} {1e3 * (time.perf_counter() - t) / n:.4f} ms")


def ev_only():
    ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, u, f, K, stream=s)


def ev_check():
    ev_only()
    ev.check_error()


def ev_norm():
    ev_only()
    halo.residual_norm(f, None, s)


def step():
    ev_only()
    halo.residual_norm(f, None, s)
    ev.check_error()


def norm_only():
    halo.residual_norm(f, None, s)


for name, b in (("evaluate queued", ev_only), ("evaluate + check_error", ev_check),
                ("evaluate + norm", ev_norm), ("bench step", step), ("norm only", norm_only)):
    run(name, b)
