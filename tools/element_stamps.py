"""Per-phase cycle breakdown of the general-path element kernel (diagnostic library built by
`make -C 4c_amd diag`, loaded through FCG_LIB=diag, counters on with FCG_STAMPS=1):
wave-uniform s_memtime deltas between the kernel's barriers, summed per workgroup, divided by the
elements the workgroups processed -> cycles of one element's workgroup in each phase.
usage: element_stamps.py [--celltype hex27] [--n 40]"""
import argparse
import importlib
import json
import os
import sys

import torch

os.environ["FCG_LIB"] = "diag"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
fcg = importlib.import_module("4c_amd").fcg
ap = argparse.ArgumentParser()
ap.add_argument("--celltype", default="hex27")
ap.add_argument("--n", type=int, default=40)
a = ap.parse_args()
ct = fcg.HEX8 if a.celltype == "hex8" else fcg.HEX27
names = ["gather", "jacobians", "n_xyz", "strain_stress", "F_n_xyz", "force_pairs_scratch"]
dev = torch.device("cuda:0")
m = fcg.BoxMesh(ct, (a.n, a.n, a.n), jitter=0.02)
os.environ["FCG_STAMPS"] = "1"
for kin in (fcg.LINEAR, fcg.TOTLAG):
    for action in (fcg.CALC_NLNSTIFF, fcg.CALC_INTERNALFORCE):
        ev = fcg.Evaluator(m, kinematics=kin, path=fcg.PATH_GENERAL)
        u = torch.from_numpy(m.u_col(1e-3 if kin == fcg.LINEAR else 5e-2)).to(dev)
        f = torch.zeros(m.n_rows, dtype=torch.float64, device=dev)
        K = torch.zeros(m.nnz, dtype=torch.float64, device=dev) if action == fcg.CALC_NLNSTIFF else None
        ev.set_timing(True)
        ev.evaluate_device(action, fcg.OVERWRITE, u, f, K)
        d = ev.diagnostics()
        ne = max(d[6], 1)
        print(json.dumps({"kin": kin, "action": action, "ms_element": ev.timing()[0],
                          "ms_assemble": ev.timing()[1], "workgroups": d[7], "elements": d[6],
                          "cycles_per_element_wg": {nm: d[i] / ne for i, nm in enumerate(names)}}))
        ev.close()
