"""CPU checks of the -m address path: the oracle against published vectors and the reference's own
target files (tests/1to32.{rmd,txt} hold the hash160 / address of puzzle keys 1..32), and the C++
host (libkhhost) against the oracle: target loading, bloom bytes, generator table, hash160."""
from __future__ import annotations

import hashlib
import json
import os
import random

import pytest

from keyhuntm1cpu_amd import khhost
from tests.helpers import endo_planted_text

GOLD = os.path.join(os.path.dirname(__file__), "golden")
N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141


def _text(name: str) -> str:
    with open(os.path.join(GOLD, "address", name)) as f:
        return f.read()


@pytest.fixture(scope="module")
def keys():
    with open(os.path.join(GOLD, "puzzle_keys.json")) as f:
        return json.load(f)


def test_oracle_sha256_ripemd160_vectors(ora):
    assert ora.sha256(b"abc").hex() == "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"
    for m in (b"", b"a" * 55, b"a" * 56, b"a" * 64, b"a" * 119, bytes(range(200))):
        assert ora.sha256(m) == hashlib.sha256(m).digest()
    # Dobbertin-Bosselaers-Preneel test vectors
    assert ora.ripemd160(b"").hex() == "9c1185a5c5e9fc54612808977ee8f548b2258d31"
    assert ora.ripemd160(b"abc").hex() == "8eb208f7e05d987a9b044a8e98c6b087f15a0bfc"
    assert ora.ripemd160(b"message digest").hex() == "5d0689ef49d2fae572b881b123a85ffa21595f36"
    assert ora.ripemd160(b"a" * 1000000).hex() == "52783243c1697bdbe16d37f97f68f08325dc1528"


def test_oracle_hash160_pinned_by_reference_files(ora, keys):
    rmd = [l.strip() for l in _text("1to32.rmd").splitlines() if l.strip()]
    adr = [l.strip() for l in _text("1to32.txt").splitlines() if l.strip()]
    for n in range(1, 33):
        k = int(keys[str(n)]["key"], 16)
        h = ora.pub_hash160(ora.pubkey(k), True)
        assert h.hex() == rmd[n - 1]
        assert ora.rmd_to_address(h) == adr[n - 1]
    # puzzle #66's solved key against tests/66.rmd / 66.txt
    h66 = ora.pub_hash160(ora.pubkey(0x2832ED74F2B5E35EE), True)
    assert h66.hex() == _text("66.rmd").strip()
    assert ora.rmd_to_address(h66) == _text("66.txt").strip()


def test_oracle_address_group_finds_puzzles(ora, keys):
    O = ora.AddrTable(_text("1to32.rmd"))
    gen = ora.AddrGen(1)
    found = []
    for g in range(64):
        _, k, _ = gen.group(O, 1 + 1024 * g, 2)
        found += k
    assert sorted(found) == sorted(int(keys[str(n)]["key"], 16) for n in range(1, 17))


def test_oracle_degenerate_group_base_512(ora):
    """Group base 512: startP = 1024 G = _2Gn, dx[512] = 0 collapses the batch inverse
    (IntGroup.cpp:36-58), so the reference cannot find puzzle #10 (514) from -b 10 (quirk)."""
    O = ora.AddrTable(_text("1to32.rmd"))
    gen = ora.AddrGen(1)
    _, k, _ = gen.group(O, 512, 2)
    assert 514 not in k
    _, k, _ = gen.group(O, 1, 2)
    assert 514 in k


@pytest.mark.parametrize("name", ["1to32.txt", "1to32.rmd", "unsolvedpuzzles.rmd", "unsolvedpuzzles.txt",
                                  "66.txt", "64.rmd"])
def test_host_targets_match_oracle(ora, name):
    text = _text(name)
    A = khhost.Addr(text, n_seq=1 << 16, threads=4)
    O = ora.AddrTable(text)
    assert b"".join(A.table()) == O.table()
    bf, bits, h = A.bloom()
    assert bits == O.bloom().bits and h == O.bloom().hashes and bf == O.bloom_bytes()


def test_host_targets_quirks(ora):
    """Invalid lines are dropped after the bloom was sized by the count of >20-char lines; a base58
    line with a wrong checksum is still accepted (keyhunt.cpp:6330-6355)."""
    good = "1BgGZ9tcN4rm9KBzDn7KprQz87SZ26SAMH"
    bad_ck = good[:-1] + ("N" if good[-1] != "N" else "M")
    text = "\n".join(["# comment line that is long enough", good, "short", bad_ck,
                      "0" * 39 + "g", "751e76e8199196d454941c45d1b3a323f1433bd6", "  " + good + "  "]) + "\n"
    A = khhost.Addr(text, n_seq=1 << 16, threads=2)
    O = ora.AddrTable(text)
    assert b"".join(A.table()) == O.table()
    assert A.bloom()[0] == O.bloom_bytes()
    assert len(A.table()) == O.n


def test_host_hash160_and_address_match_oracle(ora):
    rng = random.Random(3)
    for _ in range(200):
        k = rng.randrange(1, N)
        p = ora.pubkey(k)
        xy = khhost.pubkey(k)
        assert khhost.hash160(xy, True) == ora.pub_hash160(p, True)
        assert khhost.hash160(xy, False) == ora.pub_hash160(p, False)
        h = ora.pub_hash160(p, True)
        assert khhost.rmd_to_address(h) == ora.rmd_to_address(h)


@pytest.mark.parametrize("stride", [1, 3, 0x100000001])
def test_host_generator_matches_oracle(ora, stride):
    A = khhost.Addr(_text("66.rmd"), n_seq=1 << 16, stride=stride, gpl=4, threads=4)
    g = ora.AddrGen(stride)
    assert A.giant_table() == g.table()
    offs, gpl = A.lane_offsets()
    assert gpl == 4 and len(offs) // 64 == 16
    for m in (1, 2, 15):
        assert offs[64 * m:64 * m + 64] == ora.pubkey(m * gpl * 1024 * stride).be64()


def _many_rmd_lines(n, seed=5):
    rng = random.Random(seed)
    return "\n".join("%040x" % rng.getrandbits(160) for _ in range(n)) + "\n"


@pytest.mark.parametrize("mult", [1, 4])
def test_host_bloom_multiplier_matches_oracle(ora, mult):
    """-z (FLAGBLOOMMULTIPLIER, keyhunt.cpp:766-772): initBloomFilter sizes the target bloom for
    multiplier x items when the file holds more than 10,000 targets (6559-6576).  12,000 synthetic
    hash160 lines: the host's bloom is byte-equal to the oracle's at -z 1 and -z 4, and -z 4's is the
    oracle's bloom_init2(4 x 12,000) geometry (larger than -z 1's)."""
    text = _many_rmd_lines(12000)
    A = khhost.Addr(text, n_seq=1 << 16, threads=4, bloom_multiplier=mult)
    O = ora.AddrTable(text, bloom_multiplier=mult)
    bf, bits, h = A.bloom()
    assert bits == O.bloom().bits and h == O.bloom().hashes and bf == O.bloom_bytes()
    ref = ora.AddrTable(text, bloom_multiplier=1)
    if mult == 4:
        assert bits > ref.bloom().bits
        assert O.bloom().entries == 4 * 12000
    ref.close()
    O.close()
    A.close()


def test_host_bloom_multiplier_clamped_below_10000(ora):
    """At most 10,000 targets: the bloom is sized for 10,000 entries whatever -z says (6561-6566)."""
    text = _many_rmd_lines(500)
    a1 = khhost.Addr(text, n_seq=1 << 16, threads=2, bloom_multiplier=1)
    a4 = khhost.Addr(text, n_seq=1 << 16, threads=2, bloom_multiplier=4)
    assert a1.bloom() == a4.bloom()
    a1.close()
    a4.close()


def test_oracle_endomorphism_constants(ora):
    """-e (keyhunt.cpp:579-585): lambda*P = (beta*x, y) for the reference's literals, checked against scalar
    multiplication on G and on a random point; lambda^3 = 1 (mod n), beta^3 = 1 (mod p)."""
    import random
    N, P = ora.ORDER, ora.P
    rng = random.Random(3)
    for i in range(2):
        lam, beta = ora.endo_constants(i)
        assert pow(lam, 3, N) == 1 and pow(beta, 3, P) == 1
        for k in (1, rng.randrange(1, N)):
            a, b = ora.pubkey(k), ora.pubkey(lam * k % N)
            assert (b.x.value(), b.y.value()) == (beta * a.x.value() % P, a.y.value())
    assert ora.endo_constants(1)[0] == pow(ora.endo_constants(0)[0], 2, ora.ORDER)
    assert ora.endo_constants(1)[1] == pow(ora.endo_constants(0)[1], 2, ora.P)


@pytest.mark.parametrize("search", [0, 1, 2])
def test_oracle_endomorphism_group_recovers_planted_keys(ora, search):
    """The oracle's -e group loop (ora_addr.c; keyhunt.cpp:2646-2937) recovers exactly the planted keys
    +-lambda^e * k of its -l mode, each through the reference's sign rule; without -e only e = 0 keys of k
    itself (or n - k for compressed hashes) come back.  Pins the endomorphism branch against scalar
    multiplication (ora.pubkey), which the group loop does not use."""
    import random
    rng = random.Random(40 + search)
    base, ngroups = 0x7000000000 + 1, 4
    picks = rng.sample(range(base, base + 1024 * ngroups), 60)
    text, planted = endo_planted_text(ora, picks, search)
    O = ora.AddrTable(text)
    gen = ora.AddrGen(1)
    keys_e, keys = [], []
    for g in range(ngroups):
        keys_e += gen.group(O, base + 1024 * g, search | ora.SEARCH_ENDO)[1]
        keys += gen.group(O, base + 1024 * g, search)[1]
    want = lambda c: (search == 2) or (search == 1 and c) or (search == 0 and not c)   # noqa: E731
    assert sorted(keys_e) == sorted(K for K, c, _ in planted if want(c))
    base_only = sorted(K for K, c, e in planted if want(c) and e == 0 and (c or K < ora.ORDER // 2))
    assert sorted(keys) == base_only
    assert len(keys_e) > len(keys)


@pytest.mark.parametrize("search", [0, 1, 2])
def test_host_confirm_matches_oracle_endomorphism(ora, search):
    """The host's confirmation of every bloom hit of the oracle's -e groups (khh_addr_confirm = address_host.cpp
    confirm_hit: lambda^e * key, the sign of the hit's form) recovers exactly the oracle's keys (keyhunt.cpp:
    2789-2937), and the plain kinds 0/1/2 still recover the non -e keys."""
    import random
    rng = random.Random(50 + search)
    base, ngroups = 0x7100000000 + 1, 4
    picks = rng.sample(range(base, base + 1024 * ngroups), 60)
    text, planted = endo_planted_text(ora, picks, 10 + search)
    O = ora.AddrTable(text)
    A = khhost.Addr(text, n_seq=1024 * ngroups)
    gen = ora.AddrGen(1)
    for flag in (ora.SEARCH_ENDO, 0):
        got, ref = [], []
        for g in range(ngroups):
            hits, keys, _ = gen.group(O, base + 1024 * g, search | flag)
            ref += keys
            for t, kind in hits:
                r = A.confirm(base + 1024 * g + t, kind)
                if r is not None:
                    got.append(r[0])
                    assert r[1] == ((kind & 3) < 2)
        assert sorted(got) == sorted(ref) and ref, flag
