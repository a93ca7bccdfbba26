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


def gate_bits(lg: int, probes: int, x: int) -> list[int]:
    """Bit indices of the level-0 gate (khb_load_gate) for x: a blocked bloom of 64-bit blocks,
    block (x mod 2^32) mod 2^(lg-6); within it, for p < probes, bit ((x >> 32) mod 2^32 >> 5p) mod 32
    of 32-bit word p mod 2 (include/khbsgs.h)."""
    blk = (x & 0xFFFFFFFF) & ((1 << (lg - 6)) - 1)
    w1 = (x >> 32) & 0xFFFFFFFF
    return [64 * blk + 32 * (p & 1) + ((w1 >> (5 * p)) & 31) for p in range(probes)]


def gate_pass(gate: bytes, lg: int, probes: int, x: int) -> bool:
    return all((gate[b >> 3] >> (b & 7)) & 1 for b in gate_bits(lg, probes, x))


def endo_planted_text(ora, picks, seed):
    """Target lines for keys +-lambda^e * k (e = 0, 1, 2), compressed or not, for the keys k in picks; returns the
    text and the planted keys with their compressed flag."""
    import random
    rng = random.Random(seed)
    lams = [1] + [ora.endo_constants(i)[0] for i in range(2)]
    lines, planted = [], []
    for k in picks:
        e, neg, comp = rng.randrange(3), rng.randrange(2), rng.randrange(2) == 1
        K = lams[e] * k % ora.ORDER
        if neg:
            K = ora.ORDER - K
        lines.append(ora.pub_hash160(ora.pubkey(K), comp).hex())
        planted.append((K, comp, e))
    return "\n".join(lines) + "\n", planted
