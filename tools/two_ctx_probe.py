"""Throughput of one product session with 1, 2 or 3 contexts on the SAME GPU (each context: its own
stream, scratch and full-residency launch), puzzle #66 target, k=1, sequential chunks.
Usage: python tools/two_ctx_probe.py [chunks_total]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401
from keyhuntm1cpu_amd import khhost  # noqa: E402

total = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
t = khhost.Tables(None, int(os.environ.get("K", "1")), threads=16, gpl=4)
tgt = khhost.pubkey(0x2832ED74F2B5E35EE)
two_n = 2 * t.n_low
lo = (1 << 65) + 4 * two_n
from keyhuntm1cpu_amd import khbsgs  # noqa: E402
R = khbsgs.default_lanes(0)   # one full residency (lanes)
for nctx, lanes, cpb in ((1, 0, 1024), (1, 0, 4096), (1, 4 * R, 4096), (2, 0, 1024), (1, 0, 1024), (1, 0, 4096)):
    s = khhost.Session(t, devices=[0] * nctx, lanes=lanes, chunks_per_batch=cpb, check_threads=16)
    s.run([tgt], lo, lo + 4096 * two_n, max_chunks=2048)          # warm-up
    t0 = time.perf_counter()
    res, st = s.run([tgt], lo, lo + (total + 8192) * two_n, max_chunks=total)
    dt = time.perf_counter() - t0
    s.close()
    print(f"contexts {nctx} lanes {lanes or R} chunks/launch {cpb}: {st['giant_steps'] / dt / 1e9:.3f} G steps/s over {dt:.2f} s, "
          f"launches {st['launches']}, kernel avg {1e3 * st['kernel_s'] / max(1, st['launches']):.2f} ms",
          flush=True)
