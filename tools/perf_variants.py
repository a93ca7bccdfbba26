"""A/B timing of libkhbsgs kernel variants in ONE process (interleaved rounds, median).
Usage: python tools/perf_variants.py [lib.so ...]   (default: the product library + lib/variants/*)
Tables: product host engine, default geometry (k=1), puzzle #66 target, 256 chunks per launch."""
import glob
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402,F401
from keyhuntm1cpu_amd import khhost, LIB_DIR  # noqa: E402
from keyhuntm1cpu_amd.khbsgs import Engine, LIB_PATH  # noqa: E402

paths = sys.argv[1:] or [LIB_PATH] + sorted(glob.glob(os.path.join(LIB_DIR, "variants", "*.so")))
t = khhost.Tables(None, 1, threads=16)
bf, nb, bits, h = t.bloom_concat(1)
gsn = t.giant_table()
offs, gpl = t.lane_offsets()
tgt = khhost.pubkey(0x2832ED74F2B5E35EE)
jobs = int(os.environ.get("JOBS", "256"))
centres = b"".join(t.chunk_centre((1 << 65) + c * (1 << 45), tgt) for c in range(jobs))
engines = {}
for p in paths:
    e = Engine(0, lib_path=p)
    e.load_bloom(bf, nb, bits, h)
    e.load_giant_table(gsn)
    e.load_lane_offsets(offs, gpl)
    e.scan(centres[:64 * 8], 0, 64)
    engines[p] = e
    print(f"{os.path.basename(p)}: lanes {e.lanes()}", flush=True)
times = {p: [] for p in paths}
ref = None
for rnd in range(int(os.environ.get("ROUNDS", "3"))):
    for p, e in engines.items():
        c, d, st = e.scan(centres, 0, t.cycles)
        times[p].append(st.kernel_ms)
        if "_p" in os.path.basename(p):      # probe experiments: candidates not comparable
            continue
        s = sorted(c)
        if ref is None:
            ref = s
        assert s == ref, f"{p}: candidate set differs"
steps = jobs * t.cycles * 1024
for p in paths:
    med = statistics.median(times[p])
    print(f"{os.path.basename(p):28s} median {med:8.2f} ms  min {min(times[p]):8.2f}  {steps / med / 1e6:8.3f} G steps/s", flush=True)
