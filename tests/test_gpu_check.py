"""GPU: the second and third check on the device (khb_check) against the oracle's
bsgs_secondcheck (keyhunt.cpp:4271-4368), and the product session confirming on the device.

The device tables here come from the ORACLE's geometry (blooms, bPtable, AMP tables) and a GTable built
from the oracle's ComputePublicKey, so the comparison does not route through libkhhost."""
from __future__ import annotations

import ctypes as C
import json
import os

import pytest

from keyhuntm1cpu_amd import khhost
from keyhuntm1cpu_amd.khbsgs import Engine

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
N_GEOM = "0x1000000000"        # N = 2^36: m = 2^18, m2 = 2^13, m3 = 2^8


def _splitmix(seed):
    s = seed
    while True:
        s = (s + 0x9E3779B97F4A7C15) & (2**64 - 1)
        z = s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & (2**64 - 1)
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & (2**64 - 1)
        yield z ^ (z >> 31)


@pytest.fixture(scope="module")
def ora_tables(ora):
    bs = ora.Bsgs(N_GEOM, 1)
    # GTable: entry 256*i + b - 1 = b * 2^(8i) * G (b < 256); entry 256*i + 255 = 2^(8(i+1)) * G
    parts = []
    for i in range(32):
        for b in range(1, 257):
            parts.append(ora.pubkey(b << (8 * i)).be64())
    gt = b"".join(parts)
    bp = b"".join(v + b"\0\0" + idx.to_bytes(8, "little") for v, idx in bs.bptable())
    tabs = {"gtable": gt, "amp2": bs.amp_table(2), "amp3": bs.amp_table(3), "l2": bs.bloom_concat(2),
            "l3": bs.bloom_concat(3), "bptable": bp, "m3": bs.m3, "m_double": 2 * bs.m, "m2_double": 2 * bs.m2,
            "m3_value": bs.m3, "m3_double": 2 * bs.m3}
    yield bs, tabs
    bs.close()


def _cases(ora, bs, seed):
    """(base, a, target point, kind): planted keys across a candidate's window, the third check's
    AddDirect(P, -P) case, random candidates."""
    r = _splitmix(seed)
    m, m2, m3 = bs.m, bs.m2, bs.m3
    out = []
    for _ in range(48):
        base = next(r) | ((next(r) & 0xFFFF) << 64)
        a = next(r) % 4096
        key = base + a * 2 * m + next(r) % (2 * m + 64)
        out.append((base, a, ora.pubkey(key), "planted"))
    for _ in range(16):
        base, a = next(r), next(r) % 4096
        i2, i = next(r) % 32, next(r) % 32
        key = base + a * 2 * m + i2 * 2 * m2 + i * 2 * m3 + m3
        out.append((base, a, ora.pubkey(key), "special"))
    for _ in range(32):
        base = next(r) | (next(r) << 64) | ((next(r) >> 8) << 128)
        out.append((base, next(r) & 0xFFFFFFFF, ora.pubkey(next(r) | (next(r) << 64) | (next(r) << 128)), "random"))
    return out


def _run(ora, bs, tabs, cases):
    with Engine(0) as e:
        e.load_check_tables(**tabs)
        targets = [c[2].be64() for c in cases]
        got = e.check(targets, [(c[0], c[1], i) for i, c in enumerate(cases)])
    return got


def test_device_check_matches_oracle(ora, ora_tables):
    bs, tabs = ora_tables
    cases = _cases(ora, bs, 0x636865636b31)
    got = _run(ora, bs, tabs, cases)
    n_found = n_special = 0
    for (base, a, tgt, kind), g in zip(cases, got):
        ref = bs.secondcheck(base, a, tgt)
        assert (g["key"] if g["found"] else None) == ref, (kind, hex(base), a)
        n_found += ref is not None
        n_special += ref is not None and kind == "special"
    assert n_found >= 16 and n_special >= 8
    assert sum(g["bp_hits"] for g in got) > 0


def test_device_check_dense_blooms(ora, ora_tables):
    """Every level-2 and level-3 bit set (in the oracle's blooms too): 32 third checks per candidate,
    1024 level-3 probes and bPtable searches each."""
    bs, tabs = ora_tables
    cases = _cases(ora, bs, 0x636865636b32)[:24] + _cases(ora, bs, 0x636865636b33)[-8:]
    dense = dict(tabs)
    l2, nb2, bits2, h2 = tabs["l2"]
    l3, nb3, bits3, h3 = tabs["l3"]
    dense["l2"] = (b"\xff" * len(l2), nb2, bits2, h2)
    dense["l3"] = (b"\xff" * len(l3), nb3, bits3, h3)
    got = _run(ora, bs, dense, cases)
    saved = []
    for lvl in (2, 3):
        for i in range(256):
            b = bs.bloom(lvl, i)
            saved.append((b, C.string_at(b.bf, b.bytes)))
            C.memset(b.bf, 0xFF, b.bytes)
    try:
        for (base, a, tgt, kind), g in zip(cases, got):
            assert (g["key"] if g["found"] else None) == bs.secondcheck(base, a, tgt), (kind, hex(base), a)
        assert all(g["l2_hits"] == 32 for g in got if not g["found"])
    finally:
        for b, raw in saved:
            C.memmove(b.bf, raw, b.bytes)


def test_device_check_rejects_bad_target_index(ora_tables):
    bs, tabs = ora_tables
    with Engine(0) as e:
        e.load_check_tables(**tabs)
        with pytest.raises(Exception):
            e.check([khhost.pubkey(5)], [(0, 0, 1)])


def test_session_device_check_finds_puzzles():
    """The product session with the device check (CHECK_DEVICE): puzzles 22..28 in one multi-target run,
    every key as the host check finds it, and every candidate confirmed on the GPU."""
    with open(os.path.join(GOLD, "puzzle_keys.json")) as f:
        keys = json.load(f)
    t = khhost.Tables(hex(1 << 20), 1, threads=8)
    ns = list(range(22, 29))
    targets = [khhost.parse_pubkey(keys[str(n)]["pubkey"])[0] for n in ns]
    with khhost.Session(t) as s:
        s.set_check_mode(khhost.CHECK_DEVICE)
        res, st = s.run(targets, 1 << (ns[0] - 1), 1 << ns[-1])
    assert res == [int(keys[str(n)]["key"], 16) for n in ns]
    assert st["device_checked"] >= len(ns) and st["device_checked"] <= st["candidates"]


def test_session_device_check_ungated():
    """Without the level-0 gate every level-1 false positive reaches the check: the device confirms them
    all (auto mode moves a batch of more than 4096 candidates to the GPU) and the planted key is found."""
    t = khhost.Tables(hex(1 << 32), 1, threads=8)
    key = (1 << 50) + 0x123456789A
    with khhost.Session(t) as s:
        s.set_test_hooks(use_gate=False)
        s.set_check_mode(khhost.CHECK_DEVICE)
        res, st = s.run([khhost.pubkey(key)], 1 << 50, (1 << 50) + (1 << 40), max_chunks=4096)
    assert res == [key]
    assert 0 < st["device_checked"] <= st["candidates"]


def test_cli_check_gpu_no_gate(tmp_path):
    """keyhunt_amd --check gpu --no-gate: the reference's exact level-1 candidate stream, confirmed on the
    device; puzzle 30's known answer, the exact output lines and exit status 1."""
    import subprocess
    from keyhuntm1cpu_amd import BIN_DIR
    p30 = "030d282cf2ff536d2c42f105d0b8588821a915dc3f9a05bd98bb23af67a2e92a5b"
    (tmp_path / "30.pub").write_text(p30 + "\n")
    for extra in (["--check", "gpu", "--no-gate"], ["--check", "auto"]):
        r = subprocess.run([os.path.join(BIN_DIR, "keyhunt_amd"), "-m", "bsgs", "-f", "30.pub", "-b", "30", "-n",
                            "0x100000", "-q", "-s", "0", *extra], cwd=tmp_path, capture_output=True, text=True,
                           timeout=300)
        assert r.returncode == 1, r.stdout + r.stderr
        assert "[+] Thread Key found privkey 3d94cd64" in r.stdout and "All points were found" in r.stdout
    r = subprocess.run([os.path.join(BIN_DIR, "keyhunt_amd"), "-m", "bsgs", "-f", "30.pub", "--check", "cpu"],
                       cwd=tmp_path, capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "--check: host, gpu or auto" in r.stderr
