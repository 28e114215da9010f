"""Per-phase cycle breakdown of the structured hex8 sweep kernel (diagnostic switch FCG_STAMPS)."""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
fcg = importlib.import_module("4c_amd").fcg
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100
dev = torch.device("cuda:0")
names = ["elements", "visits", "commit"]  # commit: builds with -DFCG_SWEEP_COMMIT_STAMP
for kin in (fcg.LINEAR, fcg.TOTLAG):
    m = fcg.BoxMesh(fcg.HEX8, (n, n, n), jitter=0.1)
    u = torch.from_numpy(m.u_col(1e-3)).to(dev)
    f = torch.zeros(m.n_rows, dtype=torch.float64, device=dev)
    K = torch.zeros(m.nnz, dtype=torch.float64, device=dev)
    for stamps in ("0", "1"):
        os.environ["FCG_STAMPS"] = stamps
        ev = fcg.Evaluator(m, kinematics=kin)
        ev.set_timing(True)
        ts = []
        for _ in range(5):
            ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, u, f, K)
            ts.append(ev.timing()[0])
        for _ in range(3):
            ev.evaluate_device(fcg.CALC_INTERNALFORCE, fcg.OVERWRITE, u, f, None)
        tf = ev.timing()[0]
        d = ev.diagnostics()
        line = (f"kin={kin} stamps={stamps} nlnstiff_ms={min(ts):.3f}/{sorted(ts)[2]:.3f} "
                f"internalforce_ms={tf:.3f}")
        if d:
            tot = sum(d[:3])
            wg = d[5]
            line += " per-WG kcycles: " + " ".join(
                f"{nm}={d[i] / wg / 1e3:.1f}({100 * d[i] / tot:.0f}%)" for i, nm in enumerate(names))
        print(line, flush=True)
        ev.close()
