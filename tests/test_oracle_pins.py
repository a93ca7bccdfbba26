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
