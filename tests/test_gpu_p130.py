"""Config D on the HIP path: puzzle #130 BSGS (-f tests/130.txt -b 130), BASELINE.json configs[3].

Chunk bases >= 2^129 exercise the host's 256-bit base and centre arithmetic (keyhunt.cpp:1089-1119
range setup, 3861-3869 startP = target + (order - base - intaux) * G) on top of the same kernel:
  * two whole default-geometry chunks of the real #130 pubkey, every level-1 candidate equal to the
    oracle's (ungated), and the gated set a subset that is exactly the gate-passing part;
  * planted keys d = 2^129 + off (SURVEY.md §8d splitmix64 recipe) and one in the last chunk below
    2^130, found through the product session;
  * the CLI with -b 130 on a target file holding #130 and a planted key (sequential mode).
"""
from __future__ import annotations

import json
import os
import subprocess

import pytest

from keyhuntm1cpu_amd import BIN_DIR, khhost
from tests.helpers import gate_pass

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
LO, HI = 1 << 129, 1 << 130


def _p130() -> str:
    with open(os.path.join(GOLD, "puzzle_targets.json")) as f:
        return json.load(f)["130.txt"][0]          # tests/130.txt of the reference


def _splitmix64(seed):
    s = seed
    while True:
        s = (s + 0x9E3779B97F4A7C15) & (2**64 - 1)
        z = s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & (2**64 - 1)
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & (2**64 - 1)
        yield z ^ (z >> 31)


@pytest.fixture(scope="module")
def tables_k1():
    t = khhost.Tables(None, 1, threads=16)
    yield t
    t.close()


def test_p130_chunks_match_oracle(tables_k1, ora):
    from keyhuntm1cpu_amd.khbsgs import Engine
    xy, comp = khhost.parse_pubkey(_p130())
    assert comp
    two_n = 2 * tables_k1.n_low
    tgt = ora.parse_pubkey(_p130())[0]
    assert tgt.be64() == xy
    bases = [LO + 0x1F3A5 * two_n, HI - 2 * two_n]     # inside [2^129, 2^130), last-but-one chunk
    bs = ora.Bsgs(None, 1)
    with Engine(0) as e:
        bf, nb, bits, h = tables_k1.bloom_concat(1)
        e.load_bloom(bf, nb, bits, h)
        e.load_giant_table(tables_k1.giant_table())
        offs, gpl = tables_k1.lane_offsets()
        e.load_lane_offsets(offs, gpl)
        centres = [tables_k1.chunk_centre(b, xy) for b in bases]
        for b, c in zip(bases, centres):
            assert c == bs.chunk_start(b, tgt).be64()       # host 256-bit startP == oracle's
        got, degen, st = e.scan(b"".join(centres), 0, tables_k1.cycles)
        assert st.giant_steps == 2 * tables_k1.cycles * 1024
        gate, lg = tables_k1.gate()
        probes = tables_k1.gate_probes()
        e.load_gate(gate, lg, probes)
        gated, _, _ = e.scan(b"".join(centres), 0, tables_k1.cycles)
        exp = []
        for j, a in got:
            g0 = (a // 1024) // gpl * gpl
            xs = e.dump_x(centres[j], g0, gpl)
            xb = xs[32 * (a - g0 * 1024):32 * (a - g0 * 1024) + 32]
            if gate_pass(gate, lg, probes, int.from_bytes(xb, "big")):
                exp.append((j, a))
    assert not degen
    total = 0
    for j, b in enumerate(bases):
        ref, _, _ = bs.scan(bs.chunk_start(b, tgt), 0, bs.cycles)
        assert sorted(a for jj, a in got if jj == j) == sorted(ref), j
        total += len(ref)
    assert total >= 1
    assert sorted(gated) == sorted(exp)


def test_p130_planted_keys_session(tables_k1):
    """d = 2^129 + off (off < 2^47, §8d), found from the range start; and a key in the last chunk
    below 2^130, found from a start three chunks earlier (the -b 130 range end)."""
    two_n = 2 * tables_k1.n_low
    off = next(_splitmix64(0x6B657968756E7466)) & ((1 << 47) - 1)
    d1 = LO + off
    d2 = HI - 0x123456789
    with khhost.Session(tables_k1, devices=[0], chunks_per_batch=8) as s:
        res, st = s.run([khhost.pubkey(d1)], LO, HI)
        assert res == [d1] and st["chunks"] <= 24       # the pipeline scans up to two batches past the find
        res, st = s.run([khhost.pubkey(d2)], HI - 3 * two_n, HI)
        assert res == [d2] and st["chunks"] == 3
        assert st["giant_steps"] == 3 * tables_k1.cycles * 1024


def test_cli_b130(tmp_path):
    """keyhunt_amd -m bsgs -f 130.txt -b 130: the real #130 target plus a planted key 2^129 + off in
    the same file; sequential from 2^129, four chunks: the planted key is reported, #130 is not."""
    off = (3 << 45) + 0xABCDEF12345
    d = LO + off
    from oracle import ora
    (tmp_path / "130.txt").write_text(_p130() + "\n" + ora.pubkey_hex(d) + " # planted\n")
    exe = os.path.join(BIN_DIR, "keyhunt_amd")
    r = subprocess.run([exe, "-m", "bsgs", "-f", "130.txt", "-b", "130", "-q", "-s", "0", "--max-chunks", "4"],
                       cwd=tmp_path, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "[+] Bit Range 130" in r.stdout
    assert "[+] -- from : 0x200000000000000000000000000000000" in r.stdout
    assert "[+] -- to   : 0x400000000000000000000000000000000" in r.stdout
    assert "[+] Added 2 points from file" in r.stdout
    assert r.stdout.count("Key found privkey") == 1
    assert "[+] Thread Key found privkey %x" % d in r.stdout
    assert "End" in r.stdout
