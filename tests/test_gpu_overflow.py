"""GPU: the candidate-ring overflow contract of SURVEY.md §8b.

Every level-1 hit must reach bsgs_secondcheck (keyhunt.cpp:3944-3948 -> 4271-4368).  A launch keeps at
most khb_candidate_capacity() candidates; when it counted more, the engine (engine.cpp device_thread)
splits the batch -- by jobs, then one job's groups -- and rescans the parts ahead of new chunks.  The
candidates it then confirms must be exactly the oracle's level-1 candidates, and the device-counted
giant steps must equal the submitted work once.
"""
from __future__ import annotations

import json
import os
import random

import pytest

from keyhuntm1cpu_amd import khhost
from tests.test_gpu_scan import _l1_check

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_overflow_rescan_dense_l1_matches_oracle(ora):
    """A dense synthetic level-1 bloom (each bit set with p = 0.97: ~54 % of all x pass) over four
    -n 2^32 chunks gives ~140k candidates per batch against a 4096-entry ring: the batch is rescanned in
    parts (4 jobs -> 1 job -> group ranges of 4 groups), and the recorded candidates equal the oracle's
    L1 candidates of every x of the four chunks."""
    n_str = "0x100000000"
    t = khhost.Tables(n_str, 1, threads=16)
    bs = ora.Bsgs(n_str, 1)
    try:
        _, nb, bits, hashes = t.bloom_concat(1)
        rng = random.Random(11)
        bf = bytes(sum(1 << k for k in range(8) if rng.random() < 0.97) for _ in range(256 * nb))
        key = 0xABCDEF0123
        base0, two_n, nch = 0x3000000000000000, 1 << 33, 4
        with khhost.Session(t, chunks_per_batch=nch) as s:
            s.set_test_hooks(cand_cap=4096, use_gate=False, record=True, l1_concat=bf)
            res, st = s.run([khhost.pubkey(key)], base0, base0 + nch * two_n, max_chunks=nch)
            rec = s.recorded()
        assert res == [None]
        assert st["rescans"] > 0 and st["chunks"] == nch
        assert st["giant_steps"] == nch * t.cycles * 1024
        ref = []
        tp = ora.pubkey(key)
        for c in range(nch):
            base = base0 + c * two_n
            _, xs, _ = bs.scan(bs.chunk_start(base, tp), 0, bs.cycles, want_x=True)
            ref += [(base, a) for a in range(bs.cycles * 1024)
                    if _l1_check(bf, nb, bits, hashes, xs[32 * a:32 * a + 32], ora)]
        assert len(ref) > 100000
        assert sorted((b, a) for b, k, a in rec) == sorted(ref)
        assert st["candidates"] == len(ref)
    finally:
        bs.close()
        t.close()


def test_overflow_rescan_finds_every_key():
    """The real tables with a one-entry ring: every batch holding two or more candidates (the puzzles'
    true hits) overflows and is rescanned in parts; every key is still found, once."""
    with open(os.path.join(GOLD, "puzzle_keys.json")) as f:
        keys = json.load(f)
    t = khhost.Tables(hex(1 << 24), 1, threads=8)
    ns = list(range(26, 33))
    targets = [khhost.parse_pubkey(keys[str(n)]["pubkey"])[0] for n in ns]
    try:
        with khhost.Session(t, chunks_per_batch=16) as s:
            s.set_test_hooks(cand_cap=1, use_gate=True)
            res, st = s.run(targets, 1 << (ns[0] - 1), 1 << ns[-1])
        assert res == [int(keys[str(n)]["key"], 16) for n in ns]
        assert st["rescans"] > 0
    finally:
        t.close()
