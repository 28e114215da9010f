"""Static issue model of the structured sweep's layer loop (sweep_h8_kernel<0, true, true, 0>, the
headline kernel): the instructions of one layer per wave from the kernel's ISA (hipcc
--offload-device-only -S), the visit loop counted twice (its trip count), classified by issue
resource, against the counters' dynamic counts and the measured cycles per layer.

usage: sweep_issue_model.py kernel.s [pmc_summary.txt]

Issue costs per wave instruction on gfx950 (wave64 on a 16-lane SIMD): VALU 4 cycles (FP64 FMA
at the measured 62.7 TF/s: ~5), LDS 4 cycles of LDS-pipe issue (b64) / 8 (b128, one per 2 cycles
of 128 B/cycle), VMEM 4 cycles of TA issue (64 lanes x 8 B stores: 8 cycles at 64 B/cycle), SALU 1.
"""
import collections
import re
import sys

s = open(sys.argv[1]).read().split("\n")
st = next(i for i, l in enumerate(s) if re.match(r"^_Z\S*sweep_h8_kernelILi0ELb1ELb1ELi0E\S*:", l))
en = next(i for i in range(st, len(s)) if s[i].startswith(".Lfunc_end"))
body = s[st:en]


def label_line(pat):
    return next(i for i, l in enumerate(body) if re.match(r"^\.LBB\S+:\s*;.*" + pat, l))


# the layer loop: the depth-1 loop header whose body holds a depth-2 loop; the visit loop: depth 2
outer = [i for i, l in enumerate(body) if re.match(r"^\.LBB\S+:\s*; =>This Loop Header: Depth=1", l)][0]
outer_name = body[outer].split(":")[0]
back = max(i for i, l in enumerate(body) if re.search(r"s_branch " + re.escape(outer_name) + r"$", l))
inner_hdr = [i for i, l in enumerate(body) if "Loop Header: Depth=2" in l or re.search(r"Parent Loop \S+ Depth=1", l) and "Depth=2" in l]
d2 = [i for i, l in enumerate(body) if re.search(r"Loop: Header=\S+ Depth=2", l) or re.search(r"; =>This Loop Header: Depth=2", l)]
d2_hdr = [i for i, l in enumerate(body) if re.search(r"^\.LBB\S+:\s*;\s+Parent Loop \S+ Depth=1", l)]
# the visit loop spans from its first depth-2 block to the last one
lo2 = min(d2 + d2_hdr)
hi2 = max(i for i, l in enumerate(body) if re.search(r"Loop: Header=\S+ Depth=2", l))
# extend hi2 to the end of that block
hi2 = next(i for i in range(hi2 + 1, back) if body[i].startswith(".LBB"))


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if re.match(r"v_(fma|fmac|mul|add|sub|fma_mix)_f64", op):
        return "valu_fp64"
    if "_dpp" in op or op.startswith("v_mov_b32_dpp"):
        return "valu_dpp"
    if op.startswith("v_"):
        return "valu_other"
    if op.startswith("ds_"):
        return "lds_b128" if "b128" in op else "lds"
    if op.startswith(("global_load", "buffer_load", "flat_load", "global_atomic")):
        return "vmem_load"
    if op.startswith(("global_store", "buffer_store", "flat_store")):
        return "vmem_store"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("s_barrier"):
        return "barrier"
    if op.startswith("s_"):
        return "salu"
    return "other"


def count(lo, hi):
    c = collections.Counter()
    ops = collections.Counter()
    for l in body[lo:hi]:
        l = l.strip()
        if not l or l.startswith((".", ";", "//")) or l.endswith(":"):
            continue
        op = l.split()[0]
        c[classify(op)] += 1
        ops[op] += 1
    return c, ops


outer_c, outer_ops = count(outer, back + 1)
inner_c, inner_ops = count(lo2, hi2)
layer = collections.Counter()
for k in set(outer_c) | set(inner_c):
    layer[k] = outer_c[k] + inner_c[k]  # the visit loop once more (two trips)
ops = outer_ops + inner_ops
cost = {"valu_fp64": 4, "valu_other": 4, "valu_dpp": 4, "lds": 4, "lds_b128": 8, "vmem_load": 4,
        "vmem_store": 8, "salu": 1, "waitcnt": 1, "branch": 1, "barrier": 1, "mfma": 16, "other": 1}
print(f"layer loop: ISA lines {outer}-{back}, visit loop {lo2}-{hi2} (x2)")
print("static instructions per layer per wave (every branch taken; stage-A and emit paths some")
print("waves skip by exec mask are counted in full):")
tot_valu = 0
for k in sorted(layer, key=lambda k: -layer[k]):
    print(f"  {k:12s} {layer[k]:6d}  ~{layer[k] * cost[k]:6d} issue cycles")
    if k.startswith("valu"):
        tot_valu += layer[k]
print(f"  VALU total {tot_valu}, of which FP64 {layer['valu_fp64']} ({100 * layer['valu_fp64'] / tot_valu:.0f} %)")
print("top non-FP64 VALU opcodes:")
for op, n in sorted(((o, n) for o, n in ops.items() if classify(o) in ("valu_other", "valu_dpp")), key=lambda x: -x[1])[:16]:
    print(f"  {op:28s} {n}")
if len(sys.argv) > 2:
    pmc = {}
    for l in open(sys.argv[2]):
        m = re.match(r"^(\S+)\s+([0-9.e+]+)\s+\(n=", l)
        if m:
            pmc[m.group(1)] = float(m.group(2))
    waves = pmc["SQ_WAVES"]
    # 1M box: 625 tiles in x-y, 101 node planes over the z-segments of the launch
    layers = float(sys.argv[3]) if len(sys.argv) > 3 else 31.1
    per = lambda k: pmc[k] / waves / layers
    print(f"dynamic (counters, per wave per layer, {layers} layers per wave): VALU {per('SQ_INSTS_VALU'):.0f}"
          f" (FP64 FMA {per('SQ_INSTS_VALU_FMA_F64'):.0f}, MUL {per('SQ_INSTS_VALU_MUL_F64'):.0f},"
          f" ADD {per('SQ_INSTS_VALU_ADD_F64'):.0f}), LDS {per('SQ_INSTS_LDS'):.0f},"
          f" VMEM rd {per('SQ_INSTS_VMEM_RD'):.0f} wr {per('SQ_INSTS_VMEM_WR'):.0f}, SALU {per('SQ_INSTS_SALU'):.0f}")
    wc = pmc["SQ_WAVE_CYCLES"] / waves / layers
    print(f"wave cycles per layer {wc:.0f} (counter units); VALU active {pmc['SQ_ACTIVE_INST_VALU'] / pmc['SQ_WAVE_CYCLES']:.3f},"
          f" LDS active {pmc['SQ_ACTIVE_INST_LDS'] / pmc['SQ_WAVE_CYCLES']:.3f}, waiting {pmc['SQ_WAIT_ANY'] / pmc['SQ_WAVE_CYCLES']:.3f},"
          f" issue-waiting {pmc['SQ_WAIT_INST_ANY'] / pmc['SQ_WAVE_CYCLES']:.3f}")
