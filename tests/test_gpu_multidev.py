"""GPU: the multi-device engine of the CLI (keyhunt_amd -g 0,1,...; khhost.Session(devices=[...])).

One device thread per context pulls batches of chunks from the shared cursor, as the reference's
threads pull chunks from BSGS_CURRENT (keyhunt.cpp:3824-3844), and every thread stops once all
targets are found (keyhunt.cpp:3979-3980).  The box has one GPU, so two contexts are opened on it
(-g 0,0): they run concurrently on separate streams with their own scratch, which is all the engine
sees of a second device.
"""
from __future__ import annotations

import json
import os
import subprocess

import pytest

from keyhuntm1cpu_amd import BIN_DIR, khhost
from keyhuntm1cpu_amd.partition import n_chunks

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
P63 = "0365ec2994b8cc0a20d40dd69edfe55ca32a54bcbbaa6b0ddcff36049301a54579"
LANES = 64 * 256            # small contexts, so the 2^52-key range splits into many batches


def _cli(args, cwd):
    exe = os.path.join(BIN_DIR, "keyhunt_amd")
    return subprocess.run([exe] + args, cwd=cwd, capture_output=True, text=True, timeout=300)


def test_cli_two_contexts_puzzle63(tmp_path):
    """BSGSD.md:35-36/80 known answer through -g 0,0: found exactly once, both device threads stop,
    exit status 1 after "All points were found"."""
    (tmp_path / "63.pub").write_text(P63 + "\n")
    r = _cli(["-m", "bsgs", "-f", "63.pub", "-r", "7cce500000000000:7cce600000000000", "-n", "0x1000000000",
              "-g", "0,0", "--gpu-blocks", str(LANES // 256), "-q", "-s", "0"], tmp_path)
    assert r.returncode == 1, r.stdout + r.stderr
    assert r.stdout.count("Key found privkey") == 1
    assert "[+] Thread Key found privkey 7cce5efdaccf6808" in r.stdout
    assert "All points were found" in r.stdout
    assert (tmp_path / "KEYFOUNDKEYFOUND.txt").read_text().count("Key found privkey") == 1


def test_cli_two_contexts_device_check(tmp_path):
    """-g 0,0 --check gpu: each device thread confirms its own batches on its own context (khb_check)."""
    (tmp_path / "63.pub").write_text(P63 + "\n")
    r = _cli(["-m", "bsgs", "-f", "63.pub", "-r", "7cce500000000000:7cce600000000000", "-n", "0x1000000000",
              "-g", "0,0", "--gpu-blocks", str(LANES // 256), "--check", "gpu", "-q", "-s", "0"], tmp_path)
    assert r.returncode == 1, r.stdout + r.stderr
    assert r.stdout.count("Key found privkey") == 1
    assert "[+] Thread Key found privkey 7cce5efdaccf6808" in r.stdout


def test_session_two_contexts_two_targets():
    """Two targets in different chunks of one range, two contexts: each key reported once."""
    t = khhost.Tables("0x1000000000", 1, threads=16)     # N = 2^36: 2^37 keys per chunk
    two_n = 2 * t.n_low
    lo = 1 << 56
    k1, k2 = lo + 37 * two_n + 0x1234567, lo + 3001 * two_n + 0x89ABCDE
    with khhost.Session(t, devices=[0, 0], lanes=LANES) as s:
        res, st = s.run([khhost.pubkey(k1), khhost.pubkey(k2)], lo, lo + 4096 * two_n)
    assert res == [k1, k2]
    assert st["launches"] >= 2
    t.close()


def test_session_two_contexts_cover_range_once():
    """No key in range (BSGSD.md:90-92 style negative case): the two contexts together claim every
    chunk of the range exactly once and the device-counted giant steps are chunks x cycles x 1024."""
    with open(os.path.join(GOLD, "puzzle_targets.json")) as f:
        p125 = json.load(f)["125.txt"][0]
    xy, _ = khhost.parse_pubkey(p125)
    t = khhost.Tables("0x1000000000", 1, threads=16)
    two_n = 2 * t.n_low
    lo = 1 << 124
    hi = lo + 1000 * two_n + 12345                  # ragged end: the last chunk is claimed and scanned whole
    with khhost.Session(t, devices=[0, 0], lanes=LANES, chunks_per_batch=37) as s:
        res, st = s.run([xy], lo, hi)
    assert res == [None]
    c = n_chunks(lo, hi, two_n)
    assert st["chunks"] == c == 1001
    assert st["giant_steps"] == c * t.cycles * 1024
    assert st["launches"] == -(-c // 37)             # 28 batches between the two threads
    t.close()


def test_session_four_contexts_cover_range_once_recorded():
    """four contexts on one GPU (the engine sees four devices) over a negative range of 1,001
    chunks, without the gate and with a synthetic level-1 bloom dense enough for ~20 candidates per chunk, every
    candidate recorded after the shared host confirmation pool rejected it: every chunk base appears, no (chunk, a)
    twice, the recorded count equals the device-counted candidates, and the device-counted giant steps equal the
    range once (keyhunt.cpp:3824-3844: one shared BSGS_CURRENT)."""
    import random
    with open(os.path.join(GOLD, "puzzle_targets.json")) as f:
        p125 = json.load(f)["125.txt"][0]
    xy, _ = khhost.parse_pubkey(p125)
    t = khhost.Tables("0x1000000000", 1, threads=16)
    try:
        _, nb, bits, hashes = t.bloom_concat(1)
        rng = random.Random(21)
        bf = bytes(sum(1 << k for k in range(8) if rng.random() < 0.625) for _ in range(256 * nb))
        two_n = 2 * t.n_low
        lo = 1 << 124
        hi = lo + 1000 * two_n + 777
        with khhost.Session(t, devices=[0, 0, 0, 0], lanes=LANES, chunks_per_batch=37, check_threads=8) as s:
            s.set_test_hooks(use_gate=False, record=True, l1_concat=bf)
            res, st = s.run([xy], lo, hi)
            rec = s.recorded()
        assert res == [None]
        c = n_chunks(lo, hi, two_n)
        assert st["chunks"] == c == 1001
        assert st["giant_steps"] == c * t.cycles * 1024
        assert st["launches"] == -(-c // 37)
        pairs = [(b, a) for b, _, a in rec]
        assert len(pairs) == len(set(pairs)) == st["candidates"]
        assert {b for b, _ in pairs} == {lo + i * two_n for i in range(c)}
        assert len(pairs) > 10 * c
    finally:
        t.close()


def test_cli_four_contexts_puzzle63(tmp_path):
    """-g 0,0,0,0: four device threads on one shared chunk cursor find puzzle 63 once, all stop, exit status 1."""
    (tmp_path / "63.pub").write_text(P63 + "\n")
    r = _cli(["-m", "bsgs", "-f", "63.pub", "-r", "7cce500000000000:7cce600000000000", "-n", "0x1000000000",
              "-g", "0,0,0,0", "--gpu-blocks", str(LANES // 256), "-q", "-s", "0"], tmp_path)
    assert r.returncode == 1, r.stdout + r.stderr
    assert r.stdout.count("Key found privkey") == 1
    assert "[+] Thread Key found privkey 7cce5efdaccf6808" in r.stdout
    assert "All points were found" in r.stdout
