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


def key_block(lo: int, hi: int, two_n: int, rank: int, world: int, key: int | None = None) -> tuple[int, int]:
    """rank_range, except that the block holding `key` starts at the chunk after the key's chunk (chunks
    counted from lo): a timed scan of a solved puzzle's range then never stops early on its key."""
    start, end = rank_range(lo, hi, two_n, rank, world)
    if key is not None and start <= key < end:
        start = min(end, lo + ((key - lo) // two_n + 1) * two_n)
    return start, end


def blocks_fit(lo: int, hi: int, two_n: int, world: int, chunks_per_rank: int, key: int | None = None):
    """Every rank's (start, end, fits): fits = the rank's chunks_per_rank chunks end inside its block."""
    out = []
    for r in range(world):
        s, e = key_block(lo, hi, two_n, r, world, key)
        out.append((s, e, s + chunks_per_rank * two_n <= e))
    return out


def fit_batch(lo: int, hi: int, two_n: int, world: int, steps: int, chunks: int, fill: int,
              key: int | None = None) -> int:
    """Chunks per step for `steps` steps (warmup + timed) of every rank inside its block: `chunks` when it
    fits, else the largest multiple of `fill` (chunks that give every lane one work item) that does;
    0 when not even one item per lane fits."""
    blocks = blocks_fit(lo, hi, two_n, world, steps * chunks, key)
    if all(ok for _, _, ok in blocks):
        return chunks
    room = min((e - s) // two_n for s, e, _ in blocks) // max(1, steps)
    return (room // fill) * fill if room >= fill else 0
