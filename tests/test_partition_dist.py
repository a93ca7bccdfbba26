"""Multi-rank path on CPU: world_size-2 (and 3) gloo processes partition the -b 66 range exactly as
bench.py does; the union covers every chunk once and per-rank throughput is max-reduced."""
from __future__ import annotations

import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from keyhuntm1cpu_amd.partition import n_chunks, rank_range

LO, HI, TWO_N = 1 << 65, 1 << 66, 1 << 45


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    s, e = rank_range(LO, HI, TWO_N, rank, world)
    t = torch.tensor([float(s >> 40), float(e >> 40)], dtype=torch.float64)
    out = [torch.zeros(2, dtype=torch.float64) for _ in range(world)]
    dist.all_gather(out, t)
    m = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(m, op=dist.ReduceOp.MAX)
    dist.barrier()
    if rank == 0:
        q.put(([tuple(int(v) for v in o.tolist()) for o in out], m.item()))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_partition(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + world * 7 + os.getpid() % 1000
    mp.spawn(_worker, args=(world, port, q), nprocs=world, join=True)
    ranges, mx = q.get(timeout=60)
    assert mx == world
    ranges = [(s << 40, e << 40) for s, e in ranges]
    assert ranges[0][0] == LO and ranges[-1][1] == HI
    for (s0, e0), (s1, e1) in zip(ranges, ranges[1:]):
        assert e0 == s1
    sizes = [(e - s) // TWO_N for s, e in ranges]
    assert sum(sizes) == n_chunks(LO, HI, TWO_N) and max(sizes) - min(sizes) <= 1


def test_partition_ragged():
    for world in (1, 2, 4, 7, 8):
        rs = [rank_range(10, 10 + 5 * 64 + 3, 64, r, world) for r in range(world)]
        assert rs[0][0] == 10 and rs[-1][1] == 10 + 5 * 64 + 3
        assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))


P66_KEY = 0x2832ED74F2B5E35EE        # puzzle #66's public solution (tests/66.rmd; bench.PUZZLE66_KEY)


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_p66_static_blocks(world):
    """bench.py --workload p66 for N ranks: -b 66 split into N static blocks (keyhunt.cpp:508-527 sets
    the -b range, north_star partitions it); the key's block starts at the chunk after the key's; the
    driver's 5 warmup + 20 timed steps fit inside every block: checked at 4096 chunks per step (the
    4-wave build's batch, k = 1, 2N = 2^45), so the 3-wave product's 3072 fit as well."""
    from keyhuntm1cpu_amd.partition import blocks_fit, key_block
    chunks = (5 + 20) * 4096
    blocks = blocks_fit(LO, HI, TWO_N, world, chunks, P66_KEY)
    assert all(ok for _, _, ok in blocks)
    for r, (s, e, _) in enumerate(blocks):
        rs, re_ = rank_range(LO, HI, TWO_N, r, world)
        assert LO <= rs <= s < s + chunks * TWO_N <= e == re_ <= HI
        assert (s - LO) % TWO_N == 0
        if rs <= P66_KEY < re_:
            assert s == LO + ((P66_KEY - LO) // TWO_N + 1) * TWO_N    # right after the key's chunk
        else:
            assert s == rs
    assert sum(1 for r in range(world) if rank_range(LO, HI, TWO_N, r, world)[0] <= P66_KEY
               < rank_range(LO, HI, TWO_N, r, world)[1]) == 1
    if world == 1:   # the single-GPU line's range is unchanged from round 2: from the chunk after the key's
        assert key_block(LO, HI, TWO_N, 0, 1, P66_KEY)[0] == LO + ((P66_KEY - LO) // TWO_N + 1) * TWO_N


def test_p66_blocks_overrun_detected():
    """bench.py's default 5 + 100 steps fit one GPU (190 steps after the key's chunk) but not a 2-, 4- or
    8-way split of -b 66 (the key's block then holds 62 / 62 / 30 steps after it): the bench must refuse
    them rather than scan past the block or 2^66."""
    from keyhuntm1cpu_amd.partition import blocks_fit
    for world in (2, 4, 8):
        assert not all(ok for _, _, ok in blocks_fit(LO, HI, TWO_N, world, 105 * 4096, P66_KEY))
    assert all(ok for _, _, ok in blocks_fit(LO, HI, TWO_N, 1, 105 * 4096, P66_KEY))


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_p66_batch_shrinks_to_fit(world):
    """bench.py's auto batch for a long run: shrunk to whole work items per lane so that every rank's
    W + K steps stay inside its -b 66 block; unchanged when it fits; refused (0) below one item per lane."""
    from keyhuntm1cpu_amd.partition import blocks_fit, fit_batch
    fill = 512                                     # 262,144 lanes x 8 groups / 4096 groups per chunk
    assert fit_batch(LO, HI, TWO_N, world, 25, 8 * fill, fill, P66_KEY) == 8 * fill
    for steps in (105, 300):
        c = fit_batch(LO, HI, TWO_N, world, steps, 8 * fill, fill, P66_KEY)
        if c:
            assert c % fill == 0 and fill <= c <= 8 * fill
            assert all(ok for _, _, ok in blocks_fit(LO, HI, TWO_N, world, steps * c, P66_KEY))
            if c < 8 * fill:
                assert not all(ok for _, _, ok in blocks_fit(LO, HI, TWO_N, world, steps * (c + fill), P66_KEY))
        else:
            assert not all(ok for _, _, ok in blocks_fit(LO, HI, TWO_N, world, steps * fill, P66_KEY))
    assert fit_batch(LO, HI, TWO_N, world, 5000, 8 * fill, fill, P66_KEY) == 0


def test_p66_default_run_batches():
    """The driver's default run (100 timed + 5 warmup steps) at the 4-wave auto batch: 4,096 chunks per
    step at N = 1, shrunk to 2,048 / 2,048 / 1,024 at N = 2 / 4 / 8 (profiles/r04y measured
    those batch sizes at the same per-GPU rate)."""
    from keyhuntm1cpu_amd.partition import fit_batch
    assert [fit_batch(LO, HI, TWO_N, w, 105, 4096, 512, P66_KEY) for w in (1, 2, 4, 8)] == [4096, 2048, 2048, 1024]
