"""keyhunt's -B modes (keyhunt.cpp:227): the order in which the search claims chunk bases, from the engine's
ChunkCursor (khh_chunk_sequence), against a restatement of the reference's claim blocks under bsgs_thread:
  sequential  thread_process_bsgs          3843-3844  base = BSGS_CURRENT; BSGS_CURRENT += 2N while < end
  backward    thread_process_bsgs_backward 5122-5133  end -= 2N; base = end < start ? start : end, while end > start
  both        thread_process_bsgs_both     5383-5414  TOP (end -= 2N, clamped to BSGS_CURRENT) or BOTTOM, at random
  dance       thread_process_bsgs_dance    4837-4870  TOP, BOTTOM or a uniform base in [BSGS_CURRENT, end)
Signed big integers in the restatement (the reference's Int), unsigned in the engine."""
from __future__ import annotations

import pytest

from keyhuntm1cpu_amd import khhost


def ref_backward(start, end, two_n):
    out = []
    while end > start:
        end -= two_n
        out.append(start if end < start else end)
    return out


def ref_sequential(start, end, two_n):
    out, cur = [], start
    while cur < end:
        out.append(cur)
        cur += two_n
    return out


@pytest.mark.parametrize("start,end,two_n", [(1 << 40, (1 << 40) + 10 * (1 << 21), 1 << 21),
                                             (1 << 40, (1 << 40) + 10 * (1 << 21) + 12345, 1 << 21),
                                             (0, 7 * 1000 + 1, 1000), (5, 6, 1000), (0, 2000, 1000)])
def test_sequential_and_backward_match_reference(start, end, two_n):
    assert khhost.chunk_sequence(0, start, end, two_n) == ref_sequential(start, end, two_n)
    assert khhost.chunk_sequence(1, start, end, two_n) == ref_backward(start, end, two_n)


class MT19937_64:
    """std::mt19937_64 (the engine's side choices), for an exact restatement of both / dance."""

    def __init__(self, seed):
        self.mt = [0] * 312
        self.mt[0] = seed & (2**64 - 1)
        for i in range(1, 312):
            self.mt[i] = (6364136223846793005 * (self.mt[i - 1] ^ (self.mt[i - 1] >> 62)) + i) & (2**64 - 1)
        self.i = 312

    def __call__(self):
        if self.i >= 312:
            for k in range(312):
                y = (self.mt[k] & 0xFFFFFFFF80000000) | (self.mt[(k + 1) % 312] & 0x7FFFFFFF)
                self.mt[k] = self.mt[(k + 156) % 312] ^ (y >> 1) ^ (0xB5026F5AA96619E9 if y & 1 else 0)
            self.i = 0
        y = self.mt[self.i]
        self.i += 1
        y ^= (y >> 29) & 0x5555555555555555
        y ^= (y << 17) & 0x71D67FFFEDA60000
        y ^= (y << 37) & 0xFFF7EEE000000000
        y ^= y >> 43
        return y & (2**64 - 1)


def ref_both_dance(mode, start, end, two_n, seed):
    """keyhunt.cpp:5383-5414 (both: r = rand() % 2, 0 TOP, 1 BOTTOM) and 4837-4870 (dance: % 3, 2 = a uniform
    base in [BSGS_CURRENT, n_range_end)); the choices from the engine's generator.  Middle claims are
    returned as ("mid", lo, hi)."""
    rng, cur, top, out = MT19937_64(seed), start, end, []
    while True:
        r = rng() % (2 if mode == 2 else 3)
        if r == 0:                                                     # TOP
            if not top > cur:
                break
            top -= two_n
            out.append(cur if top < cur else top)
        elif r == 1:                                                   # BOTTOM
            if not cur < top:
                break
            out.append(cur)
            cur += two_n
        else:                                                          # dance: middle
            if not cur < top:
                break
            out.append(("mid", cur, top))
    return out


@pytest.mark.parametrize("mode", [2, 4])
@pytest.mark.parametrize("seed", [1, 2, 3, 0x6b68])
def test_both_and_dance_match_reference(mode, seed):
    start, two_n = 1 << 50, 1 << 20
    end = start + 64 * two_n + 777
    got = khhost.chunk_sequence(mode, start, end, two_n, seed=seed)
    ref = ref_both_dance(mode, start, end, two_n, seed)
    assert len(got) == len(ref)
    for g, r in zip(got, ref):
        if isinstance(r, tuple):
            assert r[1] <= g < r[2]
        else:
            assert g == r
    # every key of [start, end) lies in some claimed chunk
    reach = start
    for lo in sorted(b for b, r in zip(got, ref) if not isinstance(r, tuple)):
        if lo <= reach:
            reach = max(reach, lo + two_n)
    assert reach >= end
    if mode == 4:
        assert any(isinstance(r, tuple) for r in ref)


def test_random_is_uniform_in_range():
    start, end = 1 << 60, (1 << 60) + (1 << 40)
    seq = khhost.chunk_sequence(3, start, end, 1 << 20, cap=2000)
    assert len(seq) == 2000 and all(start <= b < end for b in seq)
    assert len(set(seq)) == 2000
