"""Baby-step table build time, host CPU (16 threads) vs GPU (khb_build_baby), for growing k at the
default -n 2^44.  Prints one JSON line per k."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402
from keyhuntm1cpu_amd import khhost  # noqa: E402

for k in [int(x) for x in (sys.argv[1:] or ["4", "16", "64"])]:
    t0 = time.time()
    g = khhost.Tables(None, k, threads=16, gpu_device=0)
    tg = time.time() - t0
    ms = g.build_ms
    m = g.m
    g.close()
    tc = None
    if k <= 64:
        t0 = time.time()
        c = khhost.Tables(None, k, threads=16)
        tc = time.time() - t0
        c.close()
    print(json.dumps({"k": k, "baby_steps": m, "gpu_total_s": round(tg, 3), "gpu_kernel_ms": round(ms, 2),
                      "cpu16_total_s": round(tc, 3) if tc else None}), flush=True)
