"""Field ops of one or more libkhbsgs builds against Python big integers on many random operands
(e.g. the KHB_NONOP build, to see whether the carry wait states are architecturally needed).
Usage: python tools/debug/hazard_check.py lib.so [lib.so ...]"""
import os
import random
import sys

sys.path.insert(0, os.getcwd())
from keyhuntm1cpu_amd.khbsgs import Engine  # noqa: E402

P = 2**256 - 2**32 - 977
rng = random.Random(11)
n = 1 << 16


def rand_fe():
    r = rng.random()
    if r < 0.1:
        return P - 1 - rng.randrange(1 << 40)
    if r < 0.2:
        return rng.randrange(1 << 64)
    return rng.randrange(P)


a = [rand_fe() for _ in range(n)]
b = [rand_fe() for _ in range(n)]
ab = b"".join(x.to_bytes(32, "big") for x in a)
bb = b"".join(x.to_bytes(32, "big") for x in b)
ops = {0: lambda x, y: x * y % P, 1: lambda x, y: x * x % P, 2: lambda x, y: (x + y) % P,
       3: lambda x, y: (x - y) % P, 4: lambda x, y: pow(x, P - 2, P)}
exp = {op: [f(a[i], b[i]) for i in range(n)] for op, f in ops.items()}
for path in sys.argv[1:]:
    with Engine(0, lanes=16384, lib_path=path) as e:
        for op in ops:
            r = e.field_op(op, ab, bb if op in (0, 2, 3) else None)
            got = [int.from_bytes(r[32 * i:32 * i + 32], "big") for i in range(n)]
            bad = sum(1 for i in range(n) if got[i] != exp[op][i])
            print(f"{os.path.basename(path)} op {op}: {bad} of {n} wrong", flush=True)
