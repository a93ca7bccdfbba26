"""Issue-cost model of a kernel loop from a gfx950 .s file (hipcc --cuda-device-only -S).

Per block of the loop [head, tail]: instruction count, VALU count, and the modelled SIMD cycles at
4 waves/SIMD using the measured per-instruction costs of profiles/r03_valu_cost.txt (16 chains,
4 waves): full-rate VOP1/VOP2 (and v_bitop3_b32) ~2.6 cycles, VOP3 / carry-writing / 64-bit ops
~4.6, v_cndmask_b32 ~21, s_nop ~1.3.
Usage: python tools/debug/walk_cost.py file.s <kernel-substring> <head-label> <tail-label>"""
import re
import sys
from collections import Counter

FULL = ("v_add_u32", "v_sub_u32", "v_subrev_u32", "v_mov_b32", "v_and_b32", "v_or_b32", "v_xor_b32", "v_not_b32",
        "v_lshlrev_b32", "v_lshrrev_b32", "v_ashrrev_i32", "v_bitop3_b32", "v_mov_b64")


def cost(op: str) -> float:
    if op.startswith("s_nop"):
        return 1.3
    if not op.startswith("v_"):
        return 0.0
    if op.startswith("v_cndmask"):
        return 21.0
    if op.split("_e32")[0].split("_e64")[0] in FULL and not op.endswith("_e64"):
        return 2.6
    return 4.6


def main():
    src, name, head, tail = sys.argv[1:5]
    lines = open(src).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\w*" + name + r"\w*:", l))
    end = next(i for i in range(start, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
    order, blocks, cur = [], {}, None
    for l in lines[start:end]:
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            cur = m.group(1); order.append(cur); blocks[cur] = []; continue
        s = l.strip()
        if cur and s and not s.startswith((";", ".")):
            blocks[cur].append(s)
    i0, i1 = order.index(head), order.index(tail)
    tot = Counter()
    for b in order[i0:i1 + 1]:
        ops = [s.split()[0] for s in blocks[b]]
        valu = sum(1 for o in ops if o.startswith("v_"))
        cyc = sum(cost(o) for o in ops)
        br = [s for s in blocks[b] if s.startswith("s_cbranch") or s.startswith("s_branch")]
        print(f"{b:12s} {len(ops):5d} instr {valu:5d} valu {cyc:8.1f} cyc  {' | '.join(br)}")
        if len(sys.argv) > 5 and b in sys.argv[5:]:
            c = Counter(ops)
            for k, v in c.most_common(40):
                print(f"      {v:5d} {k}  ({cost(k)})")
            tot.update(c)


if __name__ == "__main__":
    main()
