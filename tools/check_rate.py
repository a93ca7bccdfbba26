"""Throughput of the second/third check (bsgs_secondcheck, keyhunt.cpp:4271-4368) on the device (khb_check)
and on the host pool (Tables::secondcheck through the session's CPU path), for DESIGN.md §8.

Candidates are random (chunk base, giant step) pairs of the default k=1 geometry against one target:
the level-1 false positives an ungated scan hands the check (each runs its scalar multiplication, the 32
AMP2 additions and 32 level-2 probes; an L2 false positive adds a third check).
Usage: python tools/check_rate.py [n ...]   Prints one JSON line per n."""
import json
import os
import random
import sys
import time
from concurrent.futures import ThreadPoolExecutor

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402,F401
from keyhuntm1cpu_amd import khhost  # noqa: E402
from keyhuntm1cpu_amd.khbsgs import Engine  # noqa: E402

sizes = [int(v) for v in sys.argv[1:]] or [64, 4096, 65536]
t = khhost.Tables(None, 1, threads=16)
tgt = khhost.pubkey(0x2832ED74F2B5E35EE)
rng = random.Random(7)
with Engine(0) as e:
    e.load_check_tables(**t.check_tables())
    e.check([tgt], [(1 << 65, 0, 0)])                       # warm: code object, tables
    for n in sizes:
        cands = [((1 << 65) + rng.randrange(1 << 64) * (1 << 45), rng.randrange(4096 * 1024), 0) for _ in range(n)]
        t0 = time.perf_counter()
        got = e.check([tgt], cands)
        dt = time.perf_counter() - t0
        hn = min(n, 4096)
        with ThreadPoolExecutor(16) as ex:
            t1 = time.perf_counter()
            ref = list(ex.map(lambda c: t.secondcheck(c[0], c[1], tgt), cands[:hn]))
            dh = time.perf_counter() - t1
        assert [g["key"] for g in got[:hn]] == ref
        print(json.dumps({"candidates": n, "device_s": round(dt, 4), "device_per_s": round(n / dt, 1),
                          "host16_s_for": hn, "host16_per_s": round(hn / dh, 1),
                          "l2_hits": sum(g["l2_hits"] for g in got), "found": sum(g["found"] for g in got)}),
              flush=True)
