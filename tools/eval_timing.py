"""hipEvent timing of one evaluate (K + r, OVERWRITE) for a box mesh; prints one JSON line.
usage: eval_timing.py --celltype hex8|hex27 --kinem linear|totlag --n N [--path auto|general]"""
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
ap.add_argument("--celltype", default="hex8")
ap.add_argument("--kinem", default="linear")
ap.add_argument("--n", type=int, default=50)
ap.add_argument("--path", default="auto")
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--material", default="stvk", choices=["stvk", "neohooke"])
ap.add_argument("--action", default="nlnstiff", choices=["nlnstiff", "internalforce"])
ap.add_argument("--renumber", action="store_true", help="random node/element numbering (input-file mesh)")
a = ap.parse_args()
ct = fcg.HEX8 if a.celltype == "hex8" else fcg.HEX27
kin = fcg.LINEAR if a.kinem == "linear" else fcg.TOTLAG
path = {"auto": fcg.PATH_AUTO, "general": fcg.PATH_GENERAL, "structured": fcg.PATH_STRUCTURED,
        "gather": fcg.PATH_GATHER, "colored": fcg.PATH_COLORED}[a.path]
t0 = time.perf_counter()
m = fcg.BoxMesh(ct, (a.n, a.n, a.n), jitter=0.1 if ct == fcg.HEX8 else 0.02)
u_np = m.u_col(1e-3 if kin == fcg.LINEAR else 5e-2)
if a.renumber:
    m = fcg.Discretization.renumbered(m, seed=1)
    u_np = u_np.reshape(-1, 3)[np.random.default_rng(2).permutation(m.n_node)].ravel()
t1 = time.perf_counter()
mat = fcg.MAT_STVK if a.material == "stvk" else fcg.MAT_ELASTHYPER_COUPNEOHOOKE
ev = fcg.Evaluator(m, kinematics=kin, path=path, material=mat)
t2 = time.perf_counter()
dev = torch.device("cuda:0")
u = torch.from_numpy(np.ascontiguousarray(u_np)).to(dev)
f = torch.zeros(m.n_rows, dtype=torch.float64, device=dev)
K = torch.zeros(m.nnz, dtype=torch.float64, device=dev)
act = fcg.CALC_NLNSTIFF if a.action == "nlnstiff" else fcg.CALC_INTERNALFORCE
ev.set_timing(True)
ts = []
for _ in range(a.reps):
    ev.evaluate_device(act, fcg.OVERWRITE, u, f, K)
    ts.append(ev.timing())
ms = sorted(x[0] + x[1] for x in ts)[len(ts) // 2]
print(json.dumps({"config": f"{a.celltype}-{a.kinem}-{a.material}-{a.n}^3-{a.action}" + ("-renumbered" if a.renumber else ""), "path": int(ev.info.path),
                  "elements": m.n_ele, "nnz": m.nnz, "ms_evaluate": ms,
                  "ms_element": sorted(ts)[len(ts) // 2][0], "ms_assemble": sorted(ts)[len(ts) // 2][1],
                  "elem_per_s": m.n_ele / (ms * 1e-3), "mesh_s": t1 - t0, "create_s": t2 - t1,
                  "device_bytes": int(ev.info.device_bytes), "scratch_bytes": int(ev.info.scratch_bytes)}))
