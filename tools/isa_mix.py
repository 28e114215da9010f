"""Static instruction mix of one kernel in a hipcc --save-temps .s file (diagnostics).
usage: isa_mix.py file.s kernel-substring [line-from line-to]"""
import collections
import re
import sys

text = open(sys.argv[1]).read().split("\n")
pat = sys.argv[2]
start = next(i for i, l in enumerate(text) if re.match(r"^_Z\S*" + re.escape(pat) + r"\S*:", l))
end = next(i for i in range(start + 1, len(text)) if text[i].startswith(".Lfunc_end"))
lo, hi = (int(sys.argv[3]), int(sys.argv[4])) if len(sys.argv) > 4 else (start, end)
c = collections.Counter()
for l in text[max(lo, start):min(hi, end)]:
    l = l.strip()
    if not l or l.startswith((".", ";", "//")) or l.endswith(":"):
        continue
    c[l.split()[0]] += 1
print(f"lines {start}-{end}, {sum(c.values())} instructions")
groups = collections.Counter()
for op, n in c.items():
    groups[op.split("_")[0] + "_" + (op.split("_")[1] if "_" in op else "")] += n
for op, n in c.most_common(40):
    print(f"  {op:30s}{n}")
