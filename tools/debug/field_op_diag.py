import random, sys
sys.path.insert(0, __import__("os").getcwd())
from keyhuntm1cpu_amd.khbsgs import Engine
P = 2**256 - 2**32 - 977
rng = random.Random(1)
def rand_fe():
    r = rng.random()
    if r < 0.1: return P - 1 - rng.randrange(1 << 40)
    if r < 0.2: return rng.randrange(1 << 64)
    return rng.randrange(P)
n = 4096
a = [rand_fe() for _ in range(n)]; b = [rand_fe() for _ in range(n)]
a[0] = 0; b[1] = 0
ab = b"".join(x.to_bytes(32, "big") for x in a); bb = b"".join(x.to_bytes(32, "big") for x in b)
with Engine(0, lanes=16384) as e:
    for op, f in {0: lambda x, y: x * y % P, 1: lambda x, y: x * x % P, 2: lambda x, y: (x + y) % P, 3: lambda x, y: (x - y) % P, 4: lambda x, y: pow(x, P - 2, P)}.items():
        r = e.field_op(op, ab, bb if op in (0, 2, 3) else None)
        got = [int.from_bytes(r[32 * i:32 * i + 32], "big") for i in range(n)]
        bad = [i for i in range(n) if got[i] != f(a[i], b[i])]
        print("op", op, "bad", len(bad))
        for i in bad[:3]:
            exp = f(a[i], b[i])
            print("  i", i, "a", hex(a[i]), "b", hex(b[i]), "\n    got", hex(got[i]), "\n    exp", hex(exp), "\n    diff", hex((got[i] - exp) % P))
