"""LDS / memory instruction mix per kernel of a hipcc -S assembly file.
usage: ds_mix.py file.s [substring of the kernel symbol]"""
import re
import sys

src = open(sys.argv[1]).read()
want = sys.argv[2] if len(sys.argv) > 2 else ""
for m in re.finditer(r"^(_Z\S+):\s*;", src, re.M):
    name = m.group(1)
    if want not in name:
        continue
    body = src[m.end():src.find(".Lfunc_end", m.end())]
    c = {}
    for line in body.split("\n"):
        t = line.strip().split()
        if t and re.match(r"(ds_|global_|buffer_|s_waitcnt|s_barrier)", t[0]):
            c[t[0]] = c.get(t[0], 0) + 1
    print(name)
    for k, v in sorted(c.items(), key=lambda x: -x[1]):
        print(f"  {k:28s} {v}")
