"""Per-phase cycle split of the hex27 element kernel (fcg_hex27.hip, diagnostic switch
FCG_STAMPS=1): thread 0's s_memtime deltas per phase (barrier waits included), per element."""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
fcg = importlib.import_module("4c_amd").fcg
n = int(sys.argv[1]) if len(sys.argv) > 1 else 40
dev = torch.device("cuda:0")
names = ["top-wait", "H+geo", "G", "K-image", "barrier+store", "producer(wave3)"]
for kin in (fcg.LINEAR, fcg.TOTLAG):
    m = fcg.BoxMesh(fcg.HEX27, (n, n, n), jitter=0.02)
    u = torch.from_numpy(m.u_col(1e-3 if kin == fcg.LINEAR else 5e-2)).to(dev)
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
        d = ev.diagnostics()
        line = f"kin={kin} stamps={stamps} element_ms={sorted(ts)[2]:.3f}"
        if d:
            # consumer (thread 0): phases 0-4 per iteration; producer (thread 192): phase 5
            tot = sum(d[:5])
            ne = d[7]
            line += " cycles/element: " + " ".join(
                f"{nm}={d[i] / ne:.0f}({100 * d[i] / tot:.0f}%)" for i, nm in enumerate(names[:5]))
            line += f" | {names[5]}={d[5] / ne:.0f}"
            if len(d) > 10 and d[10]:
                # overlapped schedule: thread 0's polling and row cycles per row item, and per
                # workgroup against its element cycles (all evaluates summed)
                wg = d[6]
                line += (f" | row items={d[10] / 5:.0f}/evaluate poll/item={d[8] / d[10]:.0f}"
                         f" rows/item={d[9] / d[10]:.0f} per-wg: elements={tot / wg:.0f}"
                         f" poll={d[8] / wg:.0f} rows={d[9] / wg:.0f}")
        print(line, flush=True)
        ev.close()
