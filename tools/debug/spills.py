"""Spill/reload and memory-wait report of the blocks of one kernel that hold field products
(>= MIN mads): where the register allocator spilled inside the hot loops.
Usage: python tools/debug/spills.py kernel.s <kernel-substring> [MIN]"""
import re
import sys
from collections import Counter

src, name = sys.argv[1], sys.argv[2]
mn = int(sys.argv[3]) if len(sys.argv) > 3 else 100
L = open(src).read().split("\n")
s = next(i for i, l in enumerate(L) if re.match(r"^_Z\w*" + name + r"\w*:", l))
e = next(i for i in range(s, len(L)) if L[i].startswith(".Lfunc_end"))
print([l.strip() for l in L[e:e + 80] if "NumVgprs:" in l or "ScratchSize" in l or "Occupancy" in l][:3])
blocks, order, cur = {}, [], None
for l in L[s:e]:
    m = re.match(r"^(\.LBB\w+):", l)
    if m:
        cur = m.group(1); blocks[cur] = []; order.append(cur); continue
    t = l.strip()
    if cur and t and not t.startswith((";", ".")):
        blocks[cur].append(t)
for b in order:
    c = Counter(x.split()[0] for x in blocks[b])
    if c["v_mad_u64_u32"] >= mn:
        sp = [x for x in blocks[b] if x.startswith("scratch")]
        w = [x for x in blocks[b] if x.startswith("s_waitcnt vmcnt")]
        v = sum(n for k, n in c.items() if k.startswith("v_"))
        print(b, "valu", v, "mad", c["v_mad_u64_u32"], "spill ops", len(sp), "vmcnt waits", w[:4])
