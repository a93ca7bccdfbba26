"""GPU end-to-end: the product search (libkhhost -> libkhbsgs) and the keyhunt_amd CLI against the
reference's known answers and the oracle."""
from __future__ import annotations

import json
import os
import subprocess

import pytest

from keyhuntm1cpu_amd import BIN_DIR, khhost
from tests.helpers import gate_pass

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
P63 = "0365ec2994b8cc0a20d40dd69edfe55ca32a54bcbbaa6b0ddcff36049301a54579"
P125 = "0233709eb11e0d4439a729f21c2c443dedb727528229713f0065721ba8fa46f00e"


@pytest.fixture(scope="module")
def keys():
    with open(os.path.join(GOLD, "puzzle_keys.json")) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def tables_k1():
    t = khhost.Tables(None, 1, threads=16)
    yield t
    t.close()


def test_puzzle30_known_answer():
    t = khhost.Tables("0x100000", 1, threads=8)
    xy, _ = khhost.parse_pubkey("030d282cf2ff536d2c42f105d0b8588821a915dc3f9a05bd98bb23af67a2e92a5b")
    res, st = t.search([xy], 1 << 29, 1 << 30)
    assert res == [0x3D94CD64]


def test_last_chunk_overruns_range_end():
    """a chunk is claimed while its base is below the range end
    (keyhunt.cpp:3843-3844) and then scanned whole, so a key past the end but inside the last
    claimed chunk is found; one in the next chunk is not (the scan stops after one chunk)."""
    t = khhost.Tables("0x100000", 1, threads=8)      # N = 2^20, one chunk = 2N = 2^21 keys
    start = 1 << 40
    inside, beyond = start + (1 << 21) - 1000, start + (1 << 21) + 1000
    res, st = t.search([khhost.pubkey(inside), khhost.pubkey(beyond)], start, start + 1)
    assert res == [inside, None]
    assert st["chunks"] == 1


@pytest.mark.parametrize("nexp", [20, 24, 28])
def test_puzzles_multi_target(keys, nexp):
    """All puzzles whose range fits [2^(nexp+1), 2^(nexp+8)) in one multi-target run."""
    t = khhost.Tables(hex(1 << nexp), 1, threads=8)
    ns = [n for n in range(nexp + 2, min(nexp + 9, 46))]
    targets = [khhost.parse_pubkey(keys[str(n)]["pubkey"])[0] for n in ns]
    res, st = t.search(targets, 1 << (ns[0] - 1), 1 << ns[-1])
    assert res == [int(keys[str(n)]["key"], 16) for n in ns]


def test_puzzle63_bsgsd_known_answer(tables_k1):
    xy, _ = khhost.parse_pubkey(P63)
    res, st = tables_k1.search([xy], 0x7CCE500000000000, 0x7CCE600000000000)
    assert res == [0x7CCE5EFDACCF6808]


def test_puzzle125_not_found(tables_k1):
    """BSGSD.md:90-92 negative case, on a 2^47-wide slice of the same range."""
    xy, _ = khhost.parse_pubkey(P125)
    res, st = tables_k1.search([xy], 0x4000000000000000, 0x4000800000000000)
    assert res == [None] and st["chunks"] == 4


def test_full_geometry_candidates_match_oracle(tables_k1, ora):
    """Default -n (2^44), k=1: every L1 candidate of two whole chunks (2 x 4096 groups) equals the
    oracle's (a full-size, size-independent parity check on the real bloom)."""
    from keyhuntm1cpu_amd.khbsgs import Engine
    bs = ora.Bsgs(None, 1)
    key = 0x2832ED74F2B5E35EE
    t = ora.pubkey(key)
    bases = [key - 123456789012, (1 << 65) + (5 << 45)]
    with Engine(0) as e:
        bf, nb, bits, h = tables_k1.bloom_concat(1)
        e.load_bloom(bf, nb, bits, h)
        e.load_giant_table(tables_k1.giant_table())
        offs, gpl = tables_k1.lane_offsets()
        e.load_lane_offsets(offs, gpl)
        centres = b"".join(tables_k1.chunk_centre(b, t.be64()) for b in bases)
        got, degen, st = e.scan(centres, 0, tables_k1.cycles)
    assert not degen
    for j, b in enumerate(bases):
        ref, _, _ = bs.scan(bs.chunk_start(b, t), 0, bs.cycles)
        assert sorted(a for jj, a in got if jj == j) == sorted(ref)
    # the key's chunk yields the key through the host second check
    a_hits = [a for jj, a in got if jj == 0]
    assert any(tables_k1.secondcheck(bases[0], a, t.be64()) == key for a in a_hits)


def test_random_chunks_candidates_match_oracle(tables_k1, ora):
    """Default -n (2^44), k=1: 12 jobs of seeded random (chunk base, target key) pairs over
    [2^65, 2^66), scanned in one launch; every job's L1 candidates equal the oracle's."""
    import random
    from keyhuntm1cpu_amd.khbsgs import Engine
    bs = ora.Bsgs(None, 1)
    rng = random.Random(0x6B68)
    two_n = 1 << 45
    jobs = []
    for _ in range(12):
        base = (1 << 65) + rng.randrange(1 << 20) * two_n
        jobs.append((base, ora.pubkey((1 << 65) + rng.randrange(1 << 65))))
    with Engine(0) as e:
        bf, nb, bits, h = tables_k1.bloom_concat(1)
        e.load_bloom(bf, nb, bits, h)
        e.load_giant_table(tables_k1.giant_table())
        offs, gpl = tables_k1.lane_offsets()
        e.load_lane_offsets(offs, gpl)
        centres = b"".join(tables_k1.chunk_centre(b, t.be64()) for b, t in jobs)
        got, degen, st = e.scan(centres, 0, tables_k1.cycles)
    assert not degen
    total = 0
    for j, (b, t) in enumerate(jobs):
        ref, _, _ = bs.scan(bs.chunk_start(b, t), 0, bs.cycles)
        assert sorted(a for jj, a in got if jj == j) == sorted(ref), j
        total += len(ref)
    assert total > 12                          # ~4 L1 false positives per chunk (1e-6 x 2^22 steps)


def test_full_geometry_gate(tables_k1, ora):
    """The product's level-0 gate on the real k=1 tables (2^28 bits, three bits per x in one 64-bit
    block): over two whole chunks the gated candidates are exactly the L1 candidates whose gate
    bits are set (x from the GPU dump of their group), and the key's hit survives the gate."""
    from keyhuntm1cpu_amd.khbsgs import Engine
    gate, lg = tables_k1.gate()
    probes = tables_k1.gate_probes()
    assert lg == 28 and probes == 3
    key = 0x2832ED74F2B5E35EE
    t = ora.pubkey(key)
    bases = [key - 123456789012, (1 << 65) + (5 << 45)]
    with Engine(0) as e:
        bf, nb, bits, h = tables_k1.bloom_concat(1)
        e.load_bloom(bf, nb, bits, h)
        e.load_giant_table(tables_k1.giant_table())
        offs, gpl = tables_k1.lane_offsets()
        e.load_lane_offsets(offs, gpl)
        centres = [tables_k1.chunk_centre(b, t.be64()) for b in bases]
        plain, _, _ = e.scan(b"".join(centres), 0, tables_k1.cycles)
        # the product default (KHB_GATE_STAGE1_AUTO: a 2 MiB stage-1 fold in front of the 32 MiB gate),
        # no fold, and a 4 MiB fold give the same candidates
        by_fold = {}
        for stage1 in (0, 22, 1):
            e.set_gate_stage1(stage1)
            e.load_gate(gate, lg, probes)
            by_fold[stage1], _, st = e.scan(b"".join(centres), 0, tables_k1.cycles)
        gated = by_fold[1]
        assert sorted(by_fold[0]) == sorted(by_fold[22]) == sorted(gated)
        exp = []
        for j, a in plain:
            g0 = (a // 1024) // gpl * gpl
            xs = e.dump_x(centres[j], g0, gpl)
            xb = xs[32 * (a - g0 * 1024):32 * (a - g0 * 1024) + 32]
            if gate_pass(gate, lg, probes, int.from_bytes(xb, "big")):
                exp.append((j, a))
    assert sorted(gated) == sorted(exp)
    assert any(tables_k1.secondcheck(bases[0], a, t.be64()) == key for j, a in gated if j == 0)


def _cli(args, cwd):
    exe = os.path.join(BIN_DIR, "keyhunt_amd")
    return subprocess.run([exe] + args, cwd=cwd, capture_output=True, text=True, timeout=300)


def test_cli_puzzle63(tmp_path):
    (tmp_path / "63.pub").write_text(P63 + "\n\n")
    r = _cli(["-m", "bsgs", "-f", "63.pub", "-r", "7cce500000000000:7cce600000000000", "-q", "-s", "0"], tmp_path)
    assert r.returncode == 1, r.stdout + r.stderr          # keyhunt exits 1 after "All points were found"
    assert "[+] Thread Key found privkey 7cce5efdaccf6808" in r.stdout
    assert "[+] Publickey " + P63 in r.stdout
    assert "All points were found" in r.stdout
    kf = (tmp_path / "KEYFOUNDKEYFOUND.txt").read_text()
    assert kf == f"Key found privkey 7cce5efdaccf6808\nPublickey {P63}\n"


def test_cli_multi_target_bits(tmp_path, keys):
    lines = [keys[str(n)]["pubkey"] + " # puzzle " + str(n) for n in (31, 32, 33)]
    lines.append("04" + "zz" * 64)                          # invalid line: reported, skipped
    (tmp_path / "t.txt").write_text("\n".join(lines) + "\n")
    r = _cli(["-m", "bsgs", "-f", "t.txt", "-b", "33", "-n", "0x1000000", "-q", "-s", "0"], tmp_path)
    # puzzles 31/32 lie below 2^32: only 33 is in -b 33's range
    assert "privkey " + keys["33"]["key"] in r.stdout
    assert r.returncode == 0 and "End" in r.stdout


def test_cli_rejects_bad_geometry(tmp_path):
    (tmp_path / "63.pub").write_text(P63 + "\n")
    r = _cli(["-m", "bsgs", "-f", "63.pub", "-b", "63", "-n", "0x10000"], tmp_path)    # M = 256
    assert r.returncode == 1 and "M value is not divisible by 1024" in r.stderr
    (tmp_path / "66.txt").write_text("13zb1hQbWVsc2S7ZTZnP2G4undNNpdh5so\n")
    r = _cli(["-m", "bsgs", "-f", "66.txt", "-b", "66"], tmp_path)
    assert r.returncode == 1 and "There is no valid data in the file" in r.stderr


def _splitmix64(seed):
    s = seed
    while True:
        s = (s + 0x9E3779B97F4A7C15) & (2**64 - 1)
        z = s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & (2**64 - 1)
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & (2**64 - 1)
        yield z ^ (z >> 31)


@pytest.fixture(scope="module")
def tables_k4():
    t = khhost.Tables(None, 4, threads=16)
    yield t
    t.close()


def test_k4_full_geometry_candidates_match_oracle(tables_k4, ora):
    """Config C (-k 4, default -n): 2^24 baby steps, 57.5 MiB level-1 bloom.  Every candidate of two
    whole chunks (2 x 1024 groups) equals the oracle's, and the key comes back through the second
    check at k = 4 (M3 = 16384).  The level-0 gate's candidates are exactly the L1 candidates whose
    gate bits are set (x from the GPU dump of their group), with no fold, a 16 MiB fold, the auto 32 MiB fold
    (khb_set_gate_stage1), and the stage-0 filter in front of the 32 MiB or a 16 MiB fold (khb_set_gate_stage0,
    VERDICT r5 item 3; off in the product), and still hold the key."""
    from keyhuntm1cpu_amd.khbsgs import Engine
    bs = ora.Bsgs(None, 4)
    assert bs.m == tables_k4.m == 1 << 24 and bs.cycles == tables_k4.cycles == 1024
    key = 0x2832ED74F2B5E35EE
    t = ora.pubkey(key)
    bases = [key - 987654321098, (1 << 65) + (9 << 45)]
    with Engine(0) as e:
        bf, nb, bits, h = tables_k4.bloom_concat(1)
        e.load_bloom(bf, nb, bits, h)
        e.load_giant_table(tables_k4.giant_table())
        offs, gpl = tables_k4.lane_offsets()
        e.load_lane_offsets(offs, gpl)
        centres = b"".join(tables_k4.chunk_centre(b, t.be64()) for b in bases)
        got, degen, st = e.scan(centres, 0, tables_k4.cycles)
        # the product gate at k = 4 (2^30 bits, 128 MiB) with and without its 32 MiB stage-1 fold
        gate, lg = tables_k4.gate()
        gated = {}
        # (stage1, stage0): 1 = KHB_GATE_STAGE1_AUTO (32 MiB at k = 4: the product) / KHB_GATE_STAGE0_AUTO (the 2 MiB
        # filter in front of it, kScanG2: exact, but measured slower and off by default)
        stages = ((0, 0), (24, 0), (1, 0), (1, 1), (24, 22))
        for stage1, stage0 in stages:
            e.set_gate_stage1(stage1)
            e.set_gate_stage0(stage0)
            e.load_gate(gate, lg, tables_k4.gate_probes())
            assert e.gate_stages() == 4 | (2 if stage1 else 0) | (1 if stage0 else 0), (stage1, stage0)
            gated[stage1, stage0], gdegen, _ = e.scan(centres, 0, tables_k4.cycles)
            assert not gdegen
        # exact: gated == {L1 candidate whose x passes the gate}, as test_full_geometry_gate at k = 1
        cl = [tables_k4.chunk_centre(b, t.be64()) for b in bases]
        exp = []
        for j, a in got:
            g0 = (a // 1024) // gpl * gpl
            xs = e.dump_x(cl[j], g0, gpl)
            xb = xs[32 * (a - g0 * 1024):32 * (a - g0 * 1024) + 32]
            if gate_pass(gate, lg, tables_k4.gate_probes(), int.from_bytes(xb, "big")):
                exp.append((j, a))
    for st_ in stages:
        assert sorted(gated[st_]) == sorted(exp), st_
    assert any(tables_k4.secondcheck(bases[0], a, t.be64()) == key for jj, a in gated[1, 0] if jj == 0)
    assert not degen
    for j, b in enumerate(bases):
        ref, _, _ = bs.scan(bs.chunk_start(b, t), 0, bs.cycles)
        assert sorted(a for jj, a in got if jj == j) == sorted(ref)
    a_hits = [a for jj, a in got if jj == 0]
    assert any(tables_k4.secondcheck(bases[0], a, t.be64()) == key for a in a_hits)


def test_k4_synthetic_key_search(tables_k4):
    """SURVEY.md §8d synthetic input for B/C: d = 2^65 + off, off from splitmix64 seeded
    0x6b657968756e7466 (parity-sized: off < 2^47, found within 4 chunks), sequential from 2^65."""
    off = next(_splitmix64(0x6B657968756E7466)) & ((1 << 47) - 1)
    d = (1 << 65) + off
    xy = khhost.pubkey(d)
    res, st = tables_k4.search([xy], 1 << 65, (1 << 65) + (1 << 47))
    assert res == [d]
    assert st["chunks"] <= 4


def test_cli_save_read_table_files(tmp_path):
    """-S: the first run writes keyhunt_bsgs_{4,6,2,7}_* in the working directory, the second reads
    them (no baby-step work) and finds the same key (keyhunt.cpp:1373-1613, 1881-2025)."""
    p30 = "030d282cf2ff536d2c42f105d0b8588821a915dc3f9a05bd98bb23af67a2e92a5b"
    (tmp_path / "30.pub").write_text(p30 + "\n")
    args = ["-m", "bsgs", "-f", "30.pub", "-b", "30", "-n", "0x100000", "-S", "-q", "-s", "0"]
    r1 = _cli(args, tmp_path)
    assert r1.returncode == 1, r1.stdout + r1.stderr
    assert "[+] Writing bloom filter to file keyhunt_bsgs_4_1024.blm" in r1.stdout
    assert "[+] Writing bP Table to file keyhunt_bsgs_2_1.tbl" in r1.stdout
    assert "privkey 3d94cd64" in r1.stdout
    r2 = _cli(args, tmp_path)
    assert r2.returncode == 1, r2.stdout + r2.stderr
    assert "[+] Reading bloom filter from file keyhunt_bsgs_4_1024.blm" in r2.stdout
    assert "[+] Reading bP Table from file keyhunt_bsgs_2_1.tbl" in r2.stdout
    assert "Writing" not in r2.stdout
    assert "privkey 3d94cd64" in r2.stdout


def test_random_chunk_mode_finds_the_key(keys):
    """-R (keyhunt.cpp:3824-3844 with FLAGRANDOM): every claimed chunk starts at a random key of
    [start, end) (getrandom, Random.cpp:133-145) and is scanned whole.  The range is two chunks wide
    around puzzle 30's key, so each random chunk covers it with probability ~1/2; 40 chunks find it
    (miss probability ~2^-40) and the search stops at the find."""
    t = khhost.Tables("0x100000", 1, threads=8)      # one chunk = 2N = 2^21 keys
    try:
        key = int(keys["30"]["key"], 16)
        xy = khhost.parse_pubkey(keys["30"]["pubkey"])[0]
        two_n = 1 << 21
        with khhost.Session(t, chunks_per_batch=4) as s:
            res, st = s.run([xy], key - two_n + 1, key + two_n, max_chunks=40, random_chunks=True)
        assert res == [key]
        assert 1 <= st["chunks"] <= 40
    finally:
        t.close()


@pytest.mark.parametrize("mode", ["backward", "both", "dance"])
def test_bsgs_modes_find_keys(mode):
    """keyhunt's -B backward / both / dance (keyhunt.cpp:4794-5700) through the product session: keys near
    either end of the range are found; backward reaches the key near the end in its first chunks."""
    t = khhost.Tables(hex(1 << 24), 1, threads=8)         # 2N = 2^25 keys per chunk
    two_n = 2 * t.n_low
    start = 1 << 44
    end = start + 512 * two_n
    lo_key, hi_key = start + 3 * two_n + 0x1234, end - 2 * two_n - 0x777
    with khhost.Session(t) as s:
        s.set_chunk_mode(khhost.BSGS_MODES.index(mode))
        res, st = s.run([khhost.pubkey(lo_key), khhost.pubkey(hi_key)], start, end)
    assert res == [lo_key, hi_key]
    if mode == "backward":
        # the whole range is claimed from the top; the low key is found last
        assert st["chunks"] >= 509


def test_bsgs_backward_covers_range_once():
    """-B backward over a range of 100.5 chunks with no key in it: 101 chunks claimed (the last one clamped to
    the range start, keyhunt.cpp:5124-5125), device-counted giant steps = chunks x cycles x 1024."""
    t = khhost.Tables(hex(1 << 24), 1, threads=8)
    two_n = 2 * t.n_low
    start = 1 << 45
    end = start + 100 * two_n + two_n // 2
    with khhost.Session(t) as s:
        s.set_chunk_mode(1)
        res, st = s.run([khhost.pubkey(0x123456789)], start, end)
    assert res == [None]
    assert st["chunks"] == 101
    assert st["giant_steps"] == 101 * t.cycles * 1024


def test_cli_bsgs_backward_known_answer(tmp_path):
    p30 = "030d282cf2ff536d2c42f105d0b8588821a915dc3f9a05bd98bb23af67a2e92a5b"
    (tmp_path / "30.pub").write_text(p30 + "\n")
    r = _cli(["-m", "bsgs", "-B", "backward", "-f", "30.pub", "-b", "30", "-n", "0x100000", "-q", "-s", "0"], tmp_path)
    assert r.returncode == 1, r.stdout + r.stderr
    assert "[+] Mode BSGS backward" in r.stdout and "privkey 3d94cd64" in r.stdout
    r = _cli(["-m", "bsgs", "-B", "both", "-e", "-f", "30.pub", "-b", "30"], tmp_path)
    assert r.returncode == 1 and "Endomorphism doesn't work with BSGS" in r.stderr
