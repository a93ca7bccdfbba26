"""The oracle is pinned before it is trusted: published XXH64 vectors, the bloom
sizing of the reference geometry, the puzzle pubkeys of tests/1to63_65.txt, and the reference's
documented BSGS answers (BSGSD.md:35-36/80, puzzle-30 smoke)."""
from __future__ import annotations

import json
import os

import pytest

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_xxh64_published_vectors(ora):
    assert ora.xxh64(b"", 0) == 0xEF46DB3751D8E999
    assert ora.xxh64(b"abc", 0) == 0x44BC2CF5AD770999


def test_xxh64_stripe_path_vs_python_xxhash(ora):
    """XXH64's >= 32-byte path (4-lane stripes + mergeRounds, xxhash/xxhash.h:2469-2527) is the only
    branch bloom_check takes on 32-byte x (bloom.cpp:135-136).  Pinned against the importable
    Python xxhash (libxxhash 0.8.2), independent of this repository: 10,000 random 32-byte x with
    the bloom seed and the chained seed a, and every length 0..100 for the branch edges."""
    xxhash = pytest.importorskip("xxhash")
    import random
    rng = random.Random(0x78786836)
    seed = 0x59F2815B16F81798
    for _ in range(10000):
        x = rng.randbytes(32)
        a = ora.xxh64(x, seed)
        assert a == xxhash.xxh64_intdigest(x, seed=seed), x.hex()
        assert ora.xxh64(x, a) == xxhash.xxh64_intdigest(x, seed=a), x.hex()
    for n in range(101):
        for s in (0, seed, rng.getrandbits(64)):
            d = rng.randbytes(n)
            assert ora.xxh64(d, s) == xxhash.xxh64_intdigest(d, seed=s), (n, s)


def test_bloom_bits_fixture(ora):
    """tests/golden/bloom_bits.json (made by make_bloom_bits.py with Python xxhash, not the oracle):
    the oracle's (a, b) and its 20 bit positions per x for the k=1 and k=4 level-1 geometries
    (bloom.cpp:128-156: bit i = (a + b*i) mod bits)."""
    with open(os.path.join(GOLD, "bloom_bits.json")) as f:
        doc = json.load(f)
    seed = int(doc["seed"], 16)
    assert len(doc["records"]) >= 300
    for r in doc["records"]:
        x = bytes.fromhex(r["x"])
        a = ora.xxh64(x, seed)
        b = ora.xxh64(x, a)
        assert (a, b) == (int(r["a"], 16), int(r["b"], 16)), r["x"]
        for name, g in doc["geometries"].items():
            exp = [((a + b * i) & (2**64 - 1)) % g["bits"] for i in range(g["hashes"])]
            assert exp == r[name], (r["x"], name)


def test_bloom_bits_fixture_bloom_check(ora):
    """The oracle's bloom_check/bloom_add over the fixture's bits: a bloom holding exactly the fixture's
    bits for the first half of its x answers 1 for them and, for the rest, 1 iff all 20 of its bits
    are among those set (computed from the fixture alone)."""
    import ctypes as C
    with open(os.path.join(GOLD, "bloom_bits.json")) as f:
        doc = json.load(f)
    recs = doc["records"]
    b = ora.Bloom()
    assert ora.lib().ora_bloom_init2(C.byref(b), 16384, 0.000001) == 0
    assert b.bits == doc["geometries"]["k1"]["bits"]
    half = len(recs) // 2
    setbits = set()
    for r in recs[:half]:
        ora.lib().ora_bloom_add(C.byref(b), bytes.fromhex(r["x"]), 32)
        setbits.update(r["k1"])
    for i, r in enumerate(recs):
        exp = 1 if all(v in setbits for v in r["k1"]) else 0
        assert ora.lib().ora_bloom_check(C.byref(b), bytes.fromhex(r["x"]), 32) == exp, i
    ora.lib().ora_bloom_free(C.byref(b))


def test_bloom_sizing(ora):
    import ctypes as C
    b = ora.Bloom()
    assert ora.lib().ora_bloom_init2(C.byref(b), 16384, 0.000001) == 0
    assert (b.bits, b.bytes, b.hashes) == (471124, 58891, 20)          # SURVEY §8 k=1 row
    ora.lib().ora_bloom_free(C.byref(b))
    assert ora.lib().ora_bloom_init2(C.byref(b), 65536, 0.000001) == 0
    assert (b.bits, b.bytes, b.hashes) == (1884499, 235563, 20)        # SURVEY §8 k=4 row
    ora.lib().ora_bloom_free(C.byref(b))


def test_puzzle_pubkeys_self_certify(ora):
    with open(os.path.join(GOLD, "puzzle_keys.json")) as f:
        pk = json.load(f)
    for n, rec in pk.items():
        assert ora.pubkey_hex(int(rec["key"], 16), True) == rec["pubkey"], n


def test_puzzle30_known_answer(ora):
    bs = ora.Bsgs("0x100000", 1)
    t, _ = ora.parse_pubkey("030d282cf2ff536d2c42f105d0b8588821a915dc3f9a05bd98bb23af67a2e92a5b")
    _, keys = bs.search([t], 1 << 29, 1 << 30)
    assert keys == [0x3D94CD64]


@pytest.mark.slow
def test_puzzle63_known_answer(ora):
    bs = ora.Bsgs(None, 1)
    t, _ = ora.parse_pubkey("0365ec2994b8cc0a20d40dd69edfe55ca32a54bcbbaa6b0ddcff36049301a54579")
    _, keys = bs.search([t], 0x7CCE500000000000, 0x7CCE600000000000)
    assert keys == [0x7CCE5EFDACCF6808]


def test_check_vectors_reproduce_from_oracle(ora):
    """tests/golden/check_vectors.json is the oracle's bsgs_secondcheck output (make_golden.py check_vectors)."""
    import json
    import os
    with open(os.path.join(os.path.dirname(__file__), "golden", "check_vectors.json")) as f:
        d = json.load(f)
    bs = ora.Bsgs(d["n"], d["k"])
    for c in d["cases"]:
        t = ora.parse_pubkey("04" + c["target"])[0]
        got = bs.secondcheck(int(c["base"], 16), c["a"], t)
        assert (hex(got) if got is not None else None) == c["found"], c
