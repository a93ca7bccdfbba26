#!/usr/bin/env python3
"""bench.py — BSGS giant-step throughput on puzzle #66 (BASELINE.json configs[1]: -b 66, k=1).

One step = one GPU scan batch of the product search (libkhhost -> libkhbsgs): host centres for
512 chunks, the HIP giant-step kernel over all 4096 groups of each chunk (512 x 4096 x 1024 =
2^31 giant steps: one 8-group work item per lane of a full residency; at k=4, 2048 chunks x 1024
groups), and the CPU confirmation of every level-1 candidate, pipelined exactly as the keyhunt_amd
CLI runs it.  Tables are built and resident in HBM
before the timed region.  Chunks are sequential 2N-key chunks of -b 66 starting right after the
chunk holding puzzle #66's (public) key, so the search never stops early on the find and every
rank times exactly K steps.  Multi-GPU: one process per GPU (torch.distributed.run), rank r owns
the r-th block of (W + K) x chunks consecutive chunks (weak scaling; no data-path collective:
gloo only times it).  At N x K x chunks beyond -b 66's 2^20 chunks the blocks run on past 2^66;
the work per giant step does not depend on the keys.

Prints ONE JSON line (rank 0).  See DESIGN.md §Measurement for the roofline definitions.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

# Algorithmic work per giant step, counted in 32-bit
# multiply-class lane ops of the reference algorithm: per 1024-step group 2561 field mul
# (64 products + 8 fold) + 1023 field sqr (36 + 8) + one inversion (255 sqr + 15 mul), plus two
# XXH64 of 32 bytes (22 64-bit multiplies = 66 32-bit) and two 64-bit "% bits" (4 each).
MUL_OPS, SQR_OPS = 72, 44
OPS_PER_STEP = (2561 * MUL_OPS + 1023 * SQR_OPS + 255 * SQR_OPS + 15 * MUL_OPS) / 1024.0 + 2 * 66 + 2 * 4
# Peak of the binding unit: v_mad_u64_u32 issue rate measured on MI355X by
# tools/microbench/intops2.hip at full occupancy (profiles/r01_intops2.txt).
PEAK_MULOPS_T = float(os.environ.get("KHB_PEAK_MULOPS_T", "32.04"))
HBM_PEAK_GBS = 8000.0

PUZZLE66_KEY = 0x2832ED74F2B5E35EE            # public solution; pinned to tests/66.rmd below
PUZZLE66_HASH160 = "20d45a6a762535700ce9e0b216e31994335db8a5"   # tests/66.rmd


def puzzle66_target():
    from keyhuntm1cpu_amd import khhost
    from keyhuntm1cpu_amd.hash160 import compressed_pubkey, hash160
    xy = khhost.pubkey(PUZZLE66_KEY)
    if hash160(compressed_pubkey(xy)).hex() != PUZZLE66_HASH160:
        raise SystemExit("puzzle #66 key does not match tests/66.rmd")
    return xy


def cpu_baseline(seconds: float, threads: int):
    """Oracle (plain-C restatement of thread_process_bsgs) on the host cores, same workload."""
    from oracle import ora
    bs = ora.Bsgs(None, 1, threads)
    t = ora.pubkey(PUZZLE66_KEY)
    steps, el = bs.bench(t, 1 << 65, threads, seconds)
    bs.close()
    return steps / el


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # default: >= 30 s of steady state — 100 steps x 2^34 giant steps at ~365 ms
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--chunks", type=int, default=0,
                    help="chunks (2N keys each) per step; default: the chunks that give every lane of the device "
                         "eight work items (4096 at k=1, 16384 at k=4), as the CLI's auto batch does "
                         "(engine.cpp batch_chunks)")
    ap.add_argument("--k", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch                                   # first: share torch's HIP runtime with our libraries
    import torch.distributed as dist
    ndev = torch.cuda.device_count()
    if ndev and local >= ndev:
        # more ranks than visible GPUs (a multi-rank rehearsal on a smaller box): share round-robin
        print(f"[bench] rank {rank}: LOCAL_RANK {local} >= {ndev} visible GPUs, using GPU {local % ndev}",
              file=sys.stderr, flush=True)
        local = local % ndev
    torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)

    from keyhuntm1cpu_amd import khhost
    from keyhuntm1cpu_amd.partition import rank_range
    host_threads = min(16, os.cpu_count() or 1)
    t0 = time.time()
    tables = khhost.Tables(None, args.k, threads=host_threads, gpl=4)
    t_build = time.time() - t0
    if not args.chunks:
        # >= 2^30 giant steps per step, and enough work items to give every lane one
        from keyhuntm1cpu_amd import khbsgs
        fill = -(-khbsgs.default_lanes(local) * khbsgs.groups_per_item() // tables.cycles)
        # eight work items per lane, as the CLI's auto batch (engine.cpp batch_chunks): waves take
        # items dynamically (KHB_DYN), so a deeper queue keeps every SIMD 4 waves deep until the
        # launch's last items (profiles/r01c_dyn_probe.txt)
        args.chunks = max(1, (1 << 30) // (tables.cycles * 1024), 8 * fill)
    target = puzzle66_target()
    two_n = 2 * (tables.n_low)                     # 2N keys per chunk
    key_chunk = (PUZZLE66_KEY - (1 << 65)) // two_n
    lo = (1 << 65) + (key_chunk + 1) * two_n      # -b 66, after the key's chunk
    per_rank = (args.warmup + args.steps) * args.chunks
    start, end = rank_range(lo, lo + world * per_rank * two_n, two_n, rank, world)
    sess = khhost.Session(tables, devices=[local], chunks_per_batch=args.chunks, check_threads=host_threads)

    def sync():
        torch.cuda.synchronize()

    # warmup (untimed)
    if args.warmup:
        sess.run([target], start, end, max_chunks=args.warmup * args.chunks)
    tstart = start + args.warmup * args.chunks * two_n
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    res, st = sess.run([target], tstart, end, max_chunks=args.steps * args.chunks)
    sync()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    sess.close()
    steps_done = st["giant_steps"]
    kernel_ms = 1e3 * st["kernel_s"] / max(1, st["launches"])
    tot_steps, tmax, kmax = steps_done, dt, kernel_ms
    if world > 1:
        v = torch.tensor([float(steps_done), dt, kernel_ms], dtype=torch.float64)
        s = v.clone()
        dist.all_reduce(s, op=dist.ReduceOp.SUM)
        m = v.clone()
        dist.all_reduce(m, op=dist.ReduceOp.MAX)
        tot_steps, tmax, kmax = s[0].item(), m[1].item(), m[2].item()

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return
    gsps = tot_steps / tmax
    per_launch_steps = args.chunks * tables.cycles * 1024
    if tot_steps != world * args.steps * per_launch_steps:
        print(f"[bench] WARNING: timed {tot_steps} giant steps, expected {world * args.steps * per_launch_steps}",
              file=sys.stderr, flush=True)
    achieved = OPS_PER_STEP * per_launch_steps / (kernel_ms * 1e-3) / 1e12
    roofline = {"bound": "valu", "unit": "Tops/s", "achieved": round(achieved, 3), "peak": PEAK_MULOPS_T,
                "frac": round(achieved / PEAK_MULOPS_T, 4), "traffic": None,
                "ops": "32-bit multiply-class lane ops (v_mad_u64_u32 / v_mul_lo_u32)",
                "ops_per_giant_step": round(OPS_PER_STEP, 2), "kernel": "k_giant_scan",
                "kernel_ms_avg": round(kernel_ms, 3)}
    pmc_path = os.path.join(REPO, "profiles", "pmc_latest.json")
    if os.path.exists(pmc_path):
        try:
            with open(pmc_path) as f:
                pmc = json.load(f)
            if pmc.get("chunks_per_launch") == args.chunks and pmc.get("k") == args.k:
                roofline["traffic"] = pmc.get("hbm_bytes_per_launch")
                roofline["traffic_source"] = os.path.relpath(pmc_path, REPO)
        except (OSError, ValueError):
            pass
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        c_threads = host_threads
        v = cpu_baseline(args.cpu_seconds, c_threads)
        cpu = {"value": round(v / 1e6, 4), "unit": "Mkeys/s", "cores": c_threads, "kind": "port",
               "sample": f"oracle thread_process_bsgs restatement, puzzle #66 target, chunks from 2^65, "
                         f"{args.cpu_seconds:.0f} s window on {c_threads} threads (tables built first)"}
    out = {
        "metric": "Mkeys/s (BSGS giant-steps/s) on puzzle #66 at 1/2/4/8 MI355X",
        "value": round(gsps / 1e6, 2),
        "unit": "Mkeys/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * tmax / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "real puzzle #66 pubkey (solved key, hash160 == tests/66.rmd), -b 66 range, sequential "
                "chunks from the chunk after the key's",
        "config": {"workload": "puzzle66 -m bsgs -b 66 -k %d (BASELINE configs[%s])"
                               % (args.k, {1: "1", 4: "2"}.get(args.k, "1, k varied")),
                   "n": hex(tables.n_low), "bsgs_m": tables.m, "groups_per_chunk": tables.cycles,
                   "chunks_per_step": args.chunks, "giant_steps_per_step": per_launch_steps,
                   "parallelism": "range-partition x%d" % world, "table_build_s": round(t_build, 2),
                   "ref_keys_per_s": "%.3e" % (gsps * 2 * tables.m),
                   "candidates": st["candidates"], "found": [hex(r) if r else None for r in res]},
        "roofline": roofline,
        "cpu_baseline": cpu,
    }
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
