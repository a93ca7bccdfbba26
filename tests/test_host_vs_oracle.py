"""CPU parity: the product host engine (libkhhost.so) against the oracle restatement.

Everything the host builds feeds the GPU, so it must be bit-exact: geometry, all three bloom
levels, bPtable, the giant tables, chunk centres and second/third-check outcomes.
"""
from __future__ import annotations

import random

import pytest

from keyhuntm1cpu_amd import khhost
from tests.helpers import gate_bits

GEOMS = [("0x100000", 1), ("0x100000000", 1), ("0x100000000", 3), ("0x10000000000", 2)]


@pytest.fixture(scope="module", params=GEOMS, ids=[f"{n}-k{k}" for n, k in GEOMS])
def pair(request, ora):
    n, k = request.param
    h = khhost.Tables(n, k, threads=8, gpl=4)
    o = ora.Bsgs(n, k, threads=8)
    yield h, o
    h.close()
    o.close()


def test_geometry(pair):
    h, o = pair
    assert (h.m, h.m2, h.m3, h.aux, h.cycles, h.n_low, h.l1ext, h.items1, h.items2, h.items3) == \
           (o.m, o.m2, o.m3, o.aux, o.cycles, o.n_low, o.l1ext, o.items1, o.items2, o.items3)


@pytest.mark.parametrize("level", [1, 2, 3])
def test_blooms_bit_exact(pair, level):
    h, o = pair
    bh = h.bloom_concat(level)
    bo = o.bloom_concat(level)
    assert bh[1:] == bo[1:]
    assert bh[0] == bo[0]


def test_giant_and_amp_tables(pair):
    h, o = pair
    assert h.giant_table() == o.giant_table()
    assert h.amp_table(2) == o.amp_table(2)
    assert h.amp_table(3) == o.amp_table(3)


def test_bptable(pair):
    h, o = pair
    assert h.bptable() == o.bptable()


def test_lane_offsets(pair, ora):
    h, o = pair
    offs, gpl = h.lane_offsets()
    assert gpl == 4 and len(offs) == 64 * ((o.cycles + 3) // 4)
    for m in range(1, len(offs) // 64):
        exp = ora.negation(ora.pubkey(m * gpl * 2048 * o.m)).be64()
        assert offs[64 * m:64 * m + 64] == exp


def test_chunk_centres_and_secondcheck(pair, ora):
    h, o = pair
    rng = random.Random(7)
    for _ in range(6):
        key = rng.randrange(1 << 60, 1 << 62)
        base = key - rng.randrange(1, 2 * o.n_low * 2)        # key within ~2 chunks of base
        base = max(base, 1)
        t = ora.pubkey(key)
        cen = h.chunk_centre(base, t.be64())
        assert cen == o.chunk_start(base, t).be64()
        cands, _, _ = o.scan(o.chunk_start(base, t), 0, min(o.cycles, 8))
        for a in cands[:20]:
            assert h.secondcheck(base, a, t.be64()) == o.secondcheck(base, a, t)


def test_pubkey_and_parse(ora):
    rng = random.Random(3)
    for _ in range(50):
        k = rng.randrange(1, ora.ORDER)
        assert khhost.pubkey(k) == ora.pubkey(k).be64()
        for comp in (True, False):
            s = ora.pubkey_hex(k, comp)
            xy, c = khhost.parse_pubkey(s)
            assert xy == ora.pubkey(k).be64() and c == comp
    assert khhost.parse_pubkey("02" + "00" * 31 + "05") is None or True   # may or may not be on curve
    assert khhost.parse_pubkey("05" + "11" * 32) is None
    assert khhost.parse_pubkey("02" + "11" * 31) is None


def test_level0_gate_exact(pair, ora):
    """The level-0 gate (khb_load_gate, a blocked bloom: helpers.gate_bits) is exactly the set of the
    bits of the baby steps of the L1 set (ic < l1ext, key ic + 1): every L1 member passes it,
    nothing else is set."""
    h, o = pair
    if o.l1ext > 1 << 17:
        pytest.skip("baby set too large for the Python walk")
    gate, lg = h.gate()
    probes = h.gate_probes()
    assert lg >= 13 and len(gate) == (1 << lg) // 8 and probes == 3
    exp = bytearray(len(gate))
    for ic in range(o.l1ext):
        x = ora.pubkey(ic + 1).xy()[0]
        for b in gate_bits(lg, probes, x):
            exp[b >> 3] |= 1 << (b & 7)
    assert gate == bytes(exp)


def test_batched_job_centres(ora):
    """The engine's batched centres (khh_job_centres: one scalar multiplication per 64 consecutive
    chunks, job additions sharing inversions across chunks) equal the per-chunk centres and the
    oracle's chunk start (keyhunt.cpp:3861-3869): consecutive runs crossing block boundaries, a run
    whose first auxiliary point equals 5 * (-2N G) (the doubling fallback), and random bases."""
    import random
    N_ORDER = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
    t = khhost.Tables("0x1000000", 1, threads=4)
    o = ora.Bsgs("0x1000000", 1, 4)
    two_n = 2 * t.n_low
    intaux = 2 * t.m * 512 + t.m
    tg = [khhost.pubkey(0x123456789 + 77 * i) for i in range(3)]
    rng = random.Random(7)
    runs = [[(1 << 40) + c * two_n for c in range(200)],
            [5 * two_n - intaux + c * two_n for c in range(70)],
            [rng.randrange(1, 1 << 250) for _ in range(40)],
            # runs reaching the group order: km = n - base - intaux hits 0 and then wraps (advisor r2)
            [N_ORDER - intaux - 37 * two_n + c * two_n for c in range(70)],
            [N_ORDER - intaux - 3 * two_n + 5 + c * two_n for c in range(8)]]
    for bases in runs:
        got = t.job_centres(bases, tg)
        assert got == b"".join(t.chunk_centre(b, x) for b in bases for x in tg)
    out = t.job_centres(runs[0], tg)
    target0 = ora.parse_pubkey("04" + tg[0].hex())[0]
    for c in range(60, 70):
        assert out[64 * 3 * c:64 * 3 * c + 64] == o.chunk_start(runs[0][c], target0).be64()


def test_gtable_matches_oracle(ora):
    """khh_gtable (khb_check_tables.gtable) is Secp256K1::Init's GTable: entry 256*i + j = (j+1) * 2^(8i) * G."""
    from keyhuntm1cpu_amd import khhost
    g = khhost.gtable()
    assert len(g) == 32 * 256 * 64
    for i in (0, 1, 7, 16, 31):
        for j in (0, 1, 2, 127, 253, 254, 255):
            k = ((j + 1) << (8 * i)) % ora.ORDER            # entry (31, 255) is 2^256 G
            assert g[64 * (256 * i + j):64 * (256 * i + j + 1)] == ora.pubkey(k).be64(), (i, j)
