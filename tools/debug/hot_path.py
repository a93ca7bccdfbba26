"""VALU mix along the hot path of one loop of a gfx950 kernel (.s from `hipcc --cuda-device-only -S`).

The walk's rare branches (carry propagation, x >= p canonicalisation, queue flushes) are entered when
some lane needs them: `s_cbranch_vccz L` / `s_cbranch_execz L` skip them, so the hot path takes those
branches and falls through every other conditional branch.  Starting at the loop header label, the path is
followed until it branches back to a label at or before the header (the loop's back edge).

Usage: python tools/debug/hot_path.py file.s <kernel-substring> <header-label> [-v]
Prints the instruction classes of tools/debug/bb_path.py (full-rate, half-rate, cndmask, nop) and, with -v,
every opcode count and each cndmask with the instruction before it."""
import re
import sys
from collections import Counter

sys.path.insert(0, __import__("os").path.dirname(__file__))
from bb_path import klass  # noqa: E402


def main():
    src, name, header = sys.argv[1:4]
    lines = open(src).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\w*" + name + r"\w*:", l))
    end = next(i for i in range(start, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
    body = [l.strip() for l in lines[start:end]]
    labels = {l.split(":")[0]: i for i, l in enumerate(body) if re.match(r"^\.LBB\d+_\d+:", l)}
    i = labels[header.rstrip(":")]
    h = i
    ops, cnd, seen = Counter(), [], 0
    prev = ""
    while True:
        i += 1
        seen += 1
        if seen > 200000:
            raise SystemExit("no back edge found")
        s = body[i]
        if not s or s.startswith((";", ".")):
            continue
        op = s.split()[0]
        if op.startswith("s_cbranch_vccz") or op.startswith("s_cbranch_execz") or op == "s_branch":
            tgt = s.split()[1]
            if labels[tgt] <= h:
                break
            i = labels[tgt]
            continue
        if op.startswith("s_cbranch"):
            continue
        ops[op] += 1
        if op.startswith("v_cndmask"):
            cnd.append((s, prev))
        if op.startswith("v_"):
            prev = s
    tot = Counter()
    for op, n in ops.items():
        tot[klass(op)] += n
    print("hot path", dict(tot), "valu", tot["full"] + tot["half"] + tot["cndmask"],
          "v_mad_u64_u32", ops["v_mad_u64_u32"], "cndmask_vcc", sum(1 for c, _ in cnd if c.endswith("vcc")))
    if "-v" in sys.argv:
        for k, v in ops.most_common(40):
            print(f"  {v:5d} {k}")
        for c, p in cnd:
            print(f"  {c}   <- {p}")


if __name__ == "__main__":
    main()
