"""Candidate rate and host-confirmation load of the product search (SURVEY §8(f)3 decision data).
For several geometries and target counts: giant steps/s of the pipelined session (wall), level-1
candidates that reach the host per second, and the host time one candidate's second/third check
costs (Tables.secondcheck, timed on this host), so the confirmation share of a host core follows.
Usage (GPU box): python tools/cand_rate.py > out.json"""
import json
import os
import random
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402,F401
from keyhuntm1cpu_amd import khhost  # noqa: E402

rng = random.Random(0x6B68)
rows = []
for n, k, nt, batches in ((None, 1, 1, 6), (None, 1, 16, 6), (None, 4, 16, 4), ("0x100000000", 1, 16, 6),
                          ("0x1000000", 1, 16, 6)):
    t = khhost.Tables(n, k, threads=16)
    two_n = 2 * t.n_low
    targets = [khhost.pubkey((1 << 200) + rng.randrange(1 << 100)) for _ in range(nt)]   # far from the range
    lo = 1 << 65
    with khhost.Session(t, devices=[0]) as s:
        s.run(targets, lo, lo + (1 << 80), max_chunks=1)                                  # warm-up
        # a fixed amount of work: `batches` auto-sized batches
        from keyhuntm1cpu_amd import khbsgs
        per_job = -(-t.cycles // khbsgs.groups_per_item())
        jobs = -(-8 * khbsgs.default_lanes(0) // per_job)
        chunks = max(1, min(jobs // nt, 65536)) * batches
        t0 = time.perf_counter()
        res, st = s.run(targets, lo, lo + (chunks + 1) * two_n, max_chunks=chunks)
        dt = time.perf_counter() - t0
    # host cost of one candidate's check (the reference's bsgs_secondcheck on a non-hit)
    base = lo + 12345 * two_n
    c0 = time.perf_counter()
    for a in range(200):
        t.secondcheck(base, a * 977, targets[0])
    per_check = (time.perf_counter() - c0) / 200
    row = {"n": hex(t.n_low), "k": k, "targets": nt, "chunks": chunks, "giant_steps": st["giant_steps"],
           "wall_s": round(dt, 3), "gsteps_per_s": round(st["giant_steps"] / dt / 1e9, 3),
           "candidates": st["candidates"], "cand_per_s": round(st["candidates"] / dt, 1),
           "cand_per_1e9_steps": round(st["candidates"] / st["giant_steps"] * 1e9, 3),
           "secondcheck_us": round(per_check * 1e6, 1),
           "host_core_share": round(st["candidates"] / dt * per_check, 5)}
    rows.append(row)
    print(json.dumps(row), flush=True)
    t.close()
