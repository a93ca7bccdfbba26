"""Instruction mix of the loops of one kernel in a gfx950 .s file (hipcc --cuda-device-only -S).
Usage: python tools/debug/isa_mix.py khb.s <kernel-substring>"""
import re
import sys
from collections import Counter

src, name = sys.argv[1], sys.argv[2]
lines = open(src).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\w*" + name + r"\w*:", l))
end = next(i for i in range(start, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
body = lines[start:end]
blocks, cur, order = {}, None, []
for l in body:
    m = re.match(r"^(\.LBB\w+):", l)
    if m:
        cur = m.group(1); blocks[cur] = []; order.append(cur); continue
    s = l.strip()
    if cur and s and not s.startswith((";", ".")):
        blocks[cur].append(s.split()[0])
pos = {b: i for i, b in enumerate(order)}
loops = []
for b in order:
    for ins_line in [l for l in body]:
        pass
# back edges
for i, l in enumerate(body):
    m = re.search(r"s_c?branch\w*\s+(\.LBB\w+)", l)
    if m:
        tgt = m.group(1)
        # find the block containing line i
        blk = None
        for j in range(i, -1, -1):
            mm = re.match(r"^(\.LBB\w+):", body[j])
            if mm:
                blk = mm.group(1); break
        if blk and pos.get(tgt, 1e9) <= pos[blk]:
            loops.append((tgt, blk))
def cls(op):
    if op.startswith("s_nop"): return "s_nop"
    if op.startswith(("s_", )): return "salu/ctl"
    if op.startswith(("global_", "buffer_", "scratch_", "flat_")): return "vmem:" + op.split("_")[0] + "_" + ("load" if "load" in op else "store" if "store" in op else "atomic")
    if op.startswith("ds_"): return "lds"
    if op.startswith("v_"):
        return op
    return "other"
for (h, t) in sorted(set(loops), key=lambda x: pos[x[0]]):
    bl = order[pos[h]:pos[t] + 1]
    c = Counter(cls(op) for b in bl for op in blocks[b])
    tot = sum(c.values())
    print(f"loop {h}..{t}: {len(bl)} blocks, {tot} instrs")
    for k, v in c.most_common(25):
        print(f"   {v:6d} {k}")
