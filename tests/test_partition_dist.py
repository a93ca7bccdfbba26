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
