"""Static partition of a BSGS key range across ranks (one process per GPU).

A range [lo, hi) is cut into chunks of 2N keys (keyhunt.cpp:3830-3831: BSGS_CURRENT += 2N); rank r of
W owns the contiguous chunk block [r*C/W, (r+1)*C/W) with the remainder spread over the first
ranks.  No data-path exchange is needed: each chunk is independent."""
from __future__ import annotations


def n_chunks(lo: int, hi: int, two_n: int) -> int:
    return max(0, (hi - lo + two_n - 1) // two_n)


def rank_range(lo: int, hi: int, two_n: int, rank: int, world: int) -> tuple[int, int]:
    """Key range [start, end) of rank's chunk block; end is clipped to hi for the last rank."""
    c = n_chunks(lo, hi, two_n)
    base, rem = divmod(c, world)
    first = rank * base + min(rank, rem)
    count = base + (1 if rank < rem else 0)
    start = min(hi, lo + first * two_n)
    end = min(hi, start + count * two_n)
    return start, end
