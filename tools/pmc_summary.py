"""Summarise the rocprofv3 counter passes written by tools/pmc.sh: per-dispatch averages of every
counter for kernels whose name contains a pattern (default: sweep_h8).  FETCH_SIZE is reported as
counted and x2 (gfx950 reports half the bytes; MI355X_MICROARCH.md, HBM/rocprofv3 section)."""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "sweep_h8"
vals = defaultdict(list)
meta = {}
for f in sorted(glob.glob(os.path.join(d, "p*", "*counter_collection.csv"))):
    per = defaultdict(float)
    for r in csv.DictReader(open(f)):
        if pat not in r["Kernel_Name"]:
            continue
        per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        meta = {k: r[k] for k in ("Kernel_Name", "Grid_Size", "LDS_Block_Size", "VGPR_Count",
                                   "Accum_VGPR_Count", "Scratch_Size")}
    for (_, name), v in per.items():
        vals[name].append(v)
for k, v in meta.items():
    print(f"{k}: {v}")
avg = {k: sum(v) / len(v) for k, v in vals.items()}
for k in sorted(avg):
    print(f"{k:24s} {avg[k]:.4g}  (n={len(vals[k])})")
if "FETCH_SIZE" in avg:
    print(f"{'FETCH_SIZE x2 (bytes)':24s} {2 * avg['FETCH_SIZE'] * 1024:.4g}")
if "WRITE_SIZE" in avg:
    print(f"{'WRITE_SIZE (bytes)':24s} {avg['WRITE_SIZE'] * 1024:.4g}")
if "SQ_WAVE_CYCLES" in avg and "SQ_WAIT_ANY" in avg:
    print(f"wait_any/wave_cycles     {avg['SQ_WAIT_ANY'] / avg['SQ_WAVE_CYCLES']:.3f}")
if "SQ_ACTIVE_INST_VALU" in avg and "SQ_WAVE_CYCLES" in avg:
    print(f"valu_active/wave_cycles  {avg['SQ_ACTIVE_INST_VALU'] / avg['SQ_WAVE_CYCLES']:.3f}")
if "SQ_LDS_BANK_CONFLICT" in avg and "SQ_LDS_IDX_ACTIVE" in avg:
    print(f"lds_conflict/idx_active  {avg['SQ_LDS_BANK_CONFLICT'] / avg['SQ_LDS_IDX_ACTIVE']:.3f}")
