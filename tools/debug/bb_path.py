"""VALU instruction mix along a path of basic blocks of a gfx950 kernel (.s from hipcc -S).

Basic blocks are split at labels and after every branch; a path is given as a list of labels, each
meaning the basic block that starts at that label and its fall-through successors up to (and
including) the first branch.  Usage: python tools/debug/bb_path.py file.s <kernel-substring> L1 L2 ..."""
import re
import sys
from collections import Counter

FULL = ("v_add_u32", "v_sub_u32", "v_subrev_u32", "v_mov_b32", "v_and_b32", "v_or_b32", "v_xor_b32", "v_not_b32",
        "v_lshlrev_b32", "v_lshrrev_b32", "v_ashrrev_i32", "v_bitop3_b32", "v_mov_b64")


def klass(op: str) -> str:
    if not op.startswith("v_"):
        return "nop" if op.startswith("s_nop") else "other"
    if op.startswith("v_cndmask"):
        return "cndmask"
    base = op.replace("_e32", "").replace("_e64", "")
    return "full" if base in FULL and not op.endswith("_e64") else "half"


def main():
    src, name, *labels = sys.argv[1:]
    lines = open(src).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\w*" + name + r"\w*:", l))
    end = next(i for i in range(start, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
    body = lines[start:end]
    tot = Counter()
    ops_all = Counter()
    for lab in labels:
        i = next(k for k, l in enumerate(body) if l.startswith(lab + ":")) + 1
        c = Counter()
        while i < len(body):
            s = body[i].strip()
            i += 1
            if not s or s.startswith((";", ".")):
                continue
            op = s.split()[0]
            c[klass(op)] += 1
            ops_all[op] += 1
            if op.startswith(("s_cbranch", "s_branch")):
                break
        print(lab, dict(c))
        tot.update(c)
    print("total", dict(tot), "valu", tot["full"] + tot["half"] + tot["cndmask"])
    if "-v" in sys.argv:
        for k, v in ops_all.most_common(30):
            print(f"  {v:5d} {k}")


if __name__ == "__main__":
    main()
