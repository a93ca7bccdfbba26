"""Shared helpers for the parity tests (test infrastructure)."""
from __future__ import annotations

import random

from oracle import ora

P = ora.P
N = ora.ORDER


def lane_offsets(bs: "ora.Bsgs", gpl: int, n: int) -> bytes:
    """offs[m] = (m*gpl) * _2GSn = -(m*gpl*2048*M)*G, computed with the oracle (checker-side)."""
    out = [bytes(64)]
    for m in range(1, n):
        k = m * gpl * 2048 * bs.m
        out.append(ora.negation(ora.pubkey(k)).be64())
    return b"".join(out)


def target_for_key(k: int) -> "ora.Point":
    return ora.pubkey(k)


def rand_fe(rng: random.Random) -> int:
    r = rng.random()
    if r < 0.1:
        return P - 1 - rng.randrange(1 << 40)
    if r < 0.2:
        return rng.randrange(1 << 64)
    return rng.randrange(P)
