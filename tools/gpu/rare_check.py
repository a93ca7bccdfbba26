"""Check a forced-rare-branch build (KHB_RARE_FORCE: fe_asm.hpp's carry-propagation branch taken on
every call) against Python big integers and against the product library's x dump, bit for bit.
Usage (GPU box): python tools/gpu/rare_check.py keyhuntm1cpu_amd/lib/variants/libkhbsgs_xf.so"""
import os
import random
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import torch  # noqa: E402,F401
from keyhuntm1cpu_amd import khhost  # noqa: E402
from keyhuntm1cpu_amd.khbsgs import Engine  # noqa: E402

P = 2**256 - 2**32 - 977
rng = random.Random(11)
n = 1 << 16
edges = [0, 1, 5, P - 1, 2**255, 2**64, 2**64 + 5, 2**256 - 1, 2**255 + 2**64 - 10, 2**96 - 1]
a = [rng.randrange(P) for _ in range(n)]
b = [rng.randrange(2**256) for _ in range(n)]
k = 0
for x in edges:
    for y in edges:
        a[k], b[k] = x % P, y
        k += 1
enc = lambda v: b"".join(x.to_bytes(32, "big") for x in v)  # noqa: E731
dec = lambda r: [int.from_bytes(r[32 * i:32 * i + 32], "big") for i in range(n)]  # noqa: E731
bp = [y % P for y in b]
with Engine(0, lib_path=sys.argv[1]) as e, Engine(0) as ref:
    checks = {0: (bp, lambda x, y: x * y % P), 1: (None, lambda x, y: x * x % P),
              3: (bp, lambda x, y: (x - y) % P), 5: (b, lambda x, y: (x + y) % P),
              6: (b, lambda x, y: (x * x + y) % P)}
    for op, (bv, f) in checks.items():
        got = dec(e.field_op(op, enc(a), enc(bv) if bv is not None else None))
        assert got == [f(a[i], bv[i] if bv is not None else 0) for i in range(n)], f"op {op}"
    t = khhost.Tables("0x100000000", 1, threads=8)
    for eng in (e, ref):
        bf, nb, bits, h = t.bloom_concat(1)
        eng.load_bloom(bf, nb, bits, h)
        eng.load_giant_table(t.giant_table())
        offs, gpl = t.lane_offsets()
        eng.load_lane_offsets(offs, gpl)
    tgt = khhost.pubkey(0x3000000000ABCDEF)
    c = t.chunk_centre(0x3000000000000000, tgt)
    assert e.dump_x(c, 0, t.cycles) == ref.dump_x(c, 0, t.cycles)
print(f"rare-branch build ok: 5 field ops x {n} inputs, x dump of {t.cycles} groups identical")
