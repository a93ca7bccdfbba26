"""GPU parity: libkhbsgs.so (through its C ABI) against the oracle restatement of keyhunt.cpp.

Bit-exact for everything: field ops, bloom probes, every giant-step x-coordinate, candidate sets.
"""
from __future__ import annotations

import random

import pytest

from tests.helpers import P, gate_pass, lane_offsets, rand_fe

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from keyhuntm1cpu_amd.khbsgs import Engine
    e = Engine(0, lanes=16384)
    yield e
    e.close()


@pytest.fixture(scope="module")
def bs32(ora):
    # -n 0x100000000: M = 65536, 64 groups per chunk, 1000-entry sub-blooms
    b = ora.Bsgs("0x100000000", 1)
    yield b
    b.close()


def load_tables(eng, bs, gpl):
    bf, nb, bits, h = bs.bloom_concat(1)
    eng.load_bloom(bf, nb, bits, h)
    eng.load_giant_table(bs.giant_table())
    n_off = (bs.cycles + gpl - 1) // gpl
    eng.load_lane_offsets(lane_offsets(bs, gpl, n_off), gpl)


def test_field_ops(eng):
    rng = random.Random(1)
    n = 4096
    a = [rand_fe(rng) for _ in range(n)]
    b = [rand_fe(rng) for _ in range(n)]
    a[0] = 0
    b[1] = 0
    edges = [0, 1, 2, 5, P - 1, P - 2, P - 977, 2**255, 2**256 - 2**32 - 978, 2**224 - 1, 2**32 - 1, 2**64 - 1,
             2**64, 2**64 + 5, 2**96 - 1, 2**255 + 2**64 - 10]
    # (5, 2^64): a - b + p borrows out of limb 1 (fm_sub's rare branch, KHB_RARE)
    for k, (x, y) in enumerate((x, y) for x in edges for y in edges):
        a[2 + k], b[2 + k] = x, y
    ab = b"".join(x.to_bytes(32, "big") for x in a)
    bb = b"".join(x.to_bytes(32, "big") for x in b)
    ops = {0: lambda x, y: x * y % P, 1: lambda x, y: x * x % P, 2: lambda x, y: (x + y) % P,
           3: lambda x, y: (x - y) % P, 4: lambda x, y: pow(x, P - 2, P)}
    for op, f in ops.items():
        r = eng.field_op(op, ab, bb if op in (0, 2, 3) else None)
        got = [int.from_bytes(r[32 * i:32 * i + 32], "big") for i in range(n)]
        exp = [f(a[i], b[i]) for i in range(n)]
        assert got == exp, f"field op {op}"


def test_fused_field_ops(eng):
    """The lazy add and the squaring with a fused addend (the x-only walk, KHB_FUSE) against Python
    big integers, with operands up to 2^256 - 1 where the contract allows (fe_asm.hpp)."""
    rng = random.Random(5)
    n = 4096
    lo = [0, 1, P - 1, P - 2, 2**255, 2**32 - 1, 2**255 + 2**64 - 10]  # < p
    # (2^255 + 2^64 - 10) + 2^255: the carry fold carries out of limb 1 (fm_add_lazy's rare branch)
    hi = lo + [P, P + 1, 2**256 - 1, 2**256 - 2, 2**256 - 2**32]     # < 2^256
    a = [rand_fe(rng) for _ in range(n)]
    b = [rng.randrange(2**256) for _ in range(n)]
    k = 0
    for x in hi:
        for y in hi:
            a[k], b[k] = x, y
            k += 1
    ab = b"".join(x.to_bytes(32, "big") for x in a)
    bb = b"".join(x.to_bytes(32, "big") for x in b)
    r = eng.field_op(6, ab, bb)
    got = [int.from_bytes(r[32 * i:32 * i + 32], "big") for i in range(n)]
    assert got == [(a[i] * a[i] + b[i]) % P for i in range(n)], "fm_sqr_add"
    a2 = [x if x < P else x - P for x in a]                          # lazy add needs a < p
    ab2 = b"".join(x.to_bytes(32, "big") for x in a2)
    r = eng.field_op(5, ab2, bb)
    got = [int.from_bytes(r[32 * i:32 * i + 32], "big") for i in range(n)]
    assert got == [(a2[i] + b[i]) % P for i in range(n)], "fm_add_lazy"


def test_probe_matches_oracle(eng, bs32, ora):
    load_tables(eng, bs32, 4)
    rng = random.Random(2)
    xs = []
    for i in range(1, 2001):                 # baby steps: all members -> must hit
        xs.append(ora.pubkey(i * 7 % bs32.m + 1).x.value())
    for _ in range(20000):
        xs.append(rng.randrange(P))
    raw = b"".join(x.to_bytes(32, "big") for x in xs)
    hits = eng.probe(raw)
    import ctypes as C
    for i, x in enumerate(xs):
        xb = x.to_bytes(32, "big")
        exp = ora.lib().ora_bloom_check(C.byref(bs32.bloom(1, xb[0])), xb, 32)
        assert hits[i] == (1 if exp else 0), i
    assert all(hits[:2000])


@pytest.mark.parametrize("geom", ["k1", "k4"])
def test_probe_reproduces_bloom_bits_fixture(eng, geom):
    """khb_probe against tests/golden/bloom_bits.json (Python xxhash, not the oracle):
    256 sub-blooms of the k=1 / k=4 level-1 geometry hold exactly the fixture's bit positions of the
    first half of its x, each in sub-bloom x[0] (keyhunt.cpp:3948).  The probe of every fixture x must
    answer 1 iff all 20 of its bits are set there, a fact read off the fixture alone."""
    import json
    import os
    with open(os.path.join(os.path.dirname(__file__), "golden", "bloom_bits.json")) as f:
        doc = json.load(f)
    g = doc["geometries"][geom]
    nbits, hashes = g["bits"], g["hashes"]
    nbytes = (nbits + 7) // 8
    recs = doc["records"]
    half = len(recs) // 2
    bf = bytearray(256 * nbytes)
    sets = [set() for _ in range(256)]
    for r in recs[:half]:
        sub = int(r["x"][:2], 16)
        for v in r[geom]:
            bf[sub * nbytes + (v >> 3)] |= 1 << (v & 7)
            sets[sub].add(v)
    eng.load_bloom(bytes(bf), nbytes, nbits, hashes)
    xs = b"".join(bytes.fromhex(r["x"]) for r in recs)
    hits = eng.probe(xs)
    exp = [1 if all(v in sets[int(r["x"][:2], 16)] for v in r[geom]) else 0 for r in recs]
    assert list(hits) == exp
    assert all(hits[:half])
    # every bit matters: clearing one bit of an inserted x (not shared with another) turns its probe off
    r = recs[0]
    sub = int(r["x"][:2], 16)
    v = r[geom][7]
    if sum(v in rr[geom] for rr in recs[:half] if int(rr["x"][:2], 16) == sub) == 1:
        bf[sub * nbytes + (v >> 3)] &= ~(1 << (v & 7)) & 0xFF
        eng.load_bloom(bytes(bf), nbytes, nbits, hashes)
        assert eng.probe(bytes.fromhex(r["x"]))[0] == 0


@pytest.mark.parametrize("gpl", [1, 4])
def test_dump_x_matches_oracle(eng, bs32, ora, gpl):
    load_tables(eng, bs32, gpl)
    target = ora.pubkey(0x1234567890ABCDEF)
    base = 0x1234560000000000
    start = bs32.start = bs32.chunk_start(base, target)
    _, xs_ref, _ = bs32.scan(start, 0, 8, want_x=True)
    xs = eng.dump_x(start.be64(), 0, 8)
    assert xs == xs_ref


def test_candidates_match_oracle(eng, bs32, ora):
    gpl = 4
    load_tables(eng, bs32, gpl)
    keys = [0x2000000000123457, 0x2000001000000001 + 12345, 0x20000000ABCDEF01]
    targets = [ora.pubkey(k) for k in keys]
    base0 = 0x2000000000000000
    two_n = 2 * (1 << 32)
    centres, ref = [], []
    for c in range(8):
        base = base0 + c * two_n
        for t in targets:
            st = bs32.chunk_start(base, t)
            centres.append(st.be64())
            cands, _, _ = bs32.scan(st, 0, bs32.cycles)
            ref.append(sorted(cands))
    got, degen, stats = eng.scan(b"".join(centres), 0, bs32.cycles)
    assert not degen
    assert stats.giant_steps == len(centres) * bs32.cycles * 1024
    per_job = [[] for _ in centres]
    for job, a in got:
        per_job[job].append(a)
    assert [sorted(x) for x in per_job] == ref
    assert sum(len(r) for r in ref) > 0       # the key's chunk yields true positives


def test_degenerate_group_matches_reference(eng, bs32, ora):
    """Target exactly on a window centre: dx == 0 collapses the reference's batch inverse
    (IntGroup.cpp:36-58 + IntMod.cpp:497-500); the GPU must reproduce those x values."""
    gpl = 4
    load_tables(eng, bs32, gpl)
    M = bs32.m
    base = 0x3000000000000000
    j, i = 2, 5
    key = base + 1025 * M + 2048 * j * M - 2 * M * (i + 1)
    t = ora.pubkey(key)
    st = bs32.chunk_start(base, t)
    _, xs_ref, _ = bs32.scan(st, 0, j + 1, want_x=True)
    xs = eng.dump_x(st.be64(), 0, j + 1)
    assert xs == xs_ref
    _, degen, _ = eng.scan(st.be64(), 0, bs32.cycles)
    assert (0, j) in degen


def test_candidates_ragged_lanes_match_oracle(eng, bs32, ora):
    """Diverged waves: 62 groups per job with 4 groups per lane leaves every job's last lane two
    groups short, and 35 jobs x 16 lanes = 560 items ends mid-wave.  The survivor queue must stay
    consistent while only part of a wave is active."""
    gpl = 4
    load_tables(eng, bs32, gpl)
    rng = random.Random(5)
    base0 = 0x2100000000000000
    two_n = 2 * (1 << 32)
    keys = [base0 + rng.randrange(7 * two_n) for _ in range(5)]
    targets = [ora.pubkey(k) for k in keys]
    centres, ref = [], []
    for c in range(7):
        for t in targets:
            st = bs32.chunk_start(base0 + c * two_n, t)
            centres.append(st.be64())
            cands, _, _ = bs32.scan(st, 0, 62)
            ref.append(sorted(cands))
    got, degen, stats = eng.scan(b"".join(centres), 0, 62)
    assert not degen
    assert stats.giant_steps == 35 * 62 * 1024
    per_job = [[] for _ in centres]
    for job, a in got:
        per_job[job].append(a)
    assert [sorted(x) for x in per_job] == ref
    assert sum(len(r) for r in ref) > 0


def _l1_check(bf: bytes, nb: int, bits: int, hashes: int, xb: bytes, ora) -> bool:
    """bloom_check(&bloom_bP[x[0]], x, 32) (bloom.cpp:128-156) in Python."""
    sub = bf[xb[0] * nb:(xb[0] + 1) * nb]
    a = ora.xxh64(xb, 0x59F2815B16F81798)
    b = ora.xxh64(xb, a)
    for i in range(hashes):
        p = ((a + b * i) & 0xFFFFFFFFFFFFFFFF) % bits
        if not (sub[p >> 3] >> (p & 7)) & 1:
            return False
    return True


@pytest.mark.parametrize("probes", [1, 2, 3])
def test_gate_candidates_exact(eng, bs32, ora, probes):
    """Level-0 gate (khb_load_gate): the candidates are exactly the giant steps whose x passes the
    level-1 bloom AND whose gate bits (helpers.gate_bits: one 64-bit block, `probes` bits in it)
    are all set.  A dense synthetic L1 (each bit set with p = 0.97, so ~54 % of all x pass) and a
    random gate (each bit set with p = 0.5^(1/probes), so about half of all x pass it) exercise
    both paths on every x of four chunks; without the gate the same scan returns the plain L1
    candidates, and with a stage-1 fold of the gate in front (khb_set_gate_stage1) the gated ones."""
    gpl = 4
    load_tables(eng, bs32, gpl)
    _, nb, bits, hashes = bs32.bloom_concat(1)
    rng = random.Random(7)
    bf = bytes(sum(1 << k for k in range(8) if rng.random() < 0.97) for _ in range(256 * nb))
    eng.load_bloom(bf, nb, bits, hashes)
    lg = 16
    fill = 0.5 ** (1.0 / probes)
    gate = bytes(sum(1 << k for k in range(8) if rng.random() < fill) for _ in range((1 << lg) // 8))
    centres, l1_ref, gate_ref = [], [], []
    for c in range(4):
        st = bs32.chunk_start(0x3000000000000000 + c * (1 << 33), ora.pubkey(0xABCDEF0123 + c))
        centres.append(st.be64())
        _, xs, _ = bs32.scan(st, 0, bs32.cycles, want_x=True)
        l1, gt = [], []
        for a in range(bs32.cycles * 1024):
            xb = xs[32 * a:32 * a + 32]
            if _l1_check(bf, nb, bits, hashes, xb, ora):
                l1.append(a)
                if gate_pass(gate, lg, probes, int.from_bytes(xb, "big")):
                    gt.append(a)
        l1_ref.append(l1)
        gate_ref.append(gt)
    try:
        # stage 1 = 12: the 8 KiB gate is also kept folded to 4 KiB and tested there first
        # (khb_set_gate_stage1); stage 0 = 10: a 1 KiB filter of the gate's hi words in front of that fold
        # (khb_set_gate_stage0; built for probes >= 2).  The candidates must not change.
        for use_gate, stage1, stage0, ref in ((False, 0, 0, l1_ref), (True, 0, 0, gate_ref), (True, 12, 0, gate_ref),
                                              (True, 12, 10, gate_ref)):
            eng.set_gate_stage1(stage1)
            eng.set_gate_stage0(stage0)
            eng.load_gate(gate if use_gate else None, lg, probes)
            exp_stages = (4 if use_gate else 0) | (2 if use_gate and stage1 else 0) | \
                (1 if use_gate and stage0 and probes >= 2 else 0)
            assert eng.gate_stages() == exp_stages
            got, degen, _ = eng.scan(b"".join(centres), 0, bs32.cycles)
            per_job = [[] for _ in centres]
            for job, a in got:
                per_job[job].append(a)
            assert [sorted(x) for x in per_job] == ref, (use_gate, stage1, stage0)
        assert 0.4 < sum(map(len, gate_ref)) / sum(map(len, l1_ref)) < 0.6
        assert sum(map(len, l1_ref)) > 100000
    finally:
        eng.set_gate_stage1(1)                 # KHB_GATE_STAGE1_AUTO, the library default
        eng.set_gate_stage0(0)                 # the library default: no stage 0
        eng.load_gate(None)
        load_tables(eng, bs32, gpl)
