"""Per-phase cycle breakdown of the fused hex8 kernel for both accumulation variants
(diagnostic build switches: FCG_FUSED_ACC, FCG_STAMPS)."""
import importlib
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
fcg = importlib.import_module("4c_amd").fcg
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100
m = fcg.BoxMesh(fcg.HEX8, (n, n, n), jitter=0.1)
dev = torch.device("cuda:0")
u = torch.from_numpy(m.u_col(1e-3)).to(dev)
f = torch.zeros(m.n_rows, dtype=torch.float64, device=dev)
K = torch.zeros(m.nnz, dtype=torch.float64, device=dev)
names = ["commit", "stageA", "stageB", "accum", "flush"]
for acc in ("0", "1"):
    for stamps in ("0", "1"):
        os.environ["FCG_FUSED_ACC"] = acc
        os.environ["FCG_STAMPS"] = stamps
        ev = fcg.Evaluator(m)
        ev.set_timing(True)
        reps = 5
        ts = []
        for _ in range(reps):
            ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, u, f, K)
            ts.append(ev.timing()[0])
        d = ev.diagnostics()
        line = f"acc={acc} stamps={stamps} kernel_ms={min(ts):.3f}/{sorted(ts)[len(ts)//2]:.3f}"
        if d:
            tot = sum(d[:5])
            wg = d[5]
            line += " per-WG kcycles: " + " ".join(f"{nm}={d[i]/wg/1e3:.1f}({100*d[i]/tot:.0f}%)" for i, nm in enumerate(names))
        print(line, flush=True)
        ev.close()
