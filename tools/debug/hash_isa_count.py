"""VALU instruction counts per kernel of tools/microbench/hash_isa.hip's gfx950 assembly.
Usage: python tools/debug/hash_isa_count.py hash_isa.s"""
import re
import sys
from collections import Counter

lines = open(sys.argv[1]).read().split("\n")
cur, counts = None, {}
for l in lines:
    m = re.match(r"^(_Z\w+):", l)
    if m:
        cur = m.group(1)
        counts[cur] = Counter()
        continue
    if cur and l.strip().startswith("s_endpgm"):
        cur = None
        continue
    if cur:
        m = re.match(r"^\s+(v_\w+)", l)
        if m:
            counts[cur][m.group(1)] += 1
for k, c in counts.items():
    name = re.sub(r"^_Z\d+", "", k).split("P")[0]
    top = ", ".join(f"{n} {i}" for i, n in sorted(((v, k2) for k2, v in c.items()), reverse=True)[:5])
    print(f"{name:24s} {sum(c.values()):5d} VALU   ({top})")
