"""Round-5 diagnostic: the launch epilogue's walked count in the sequences perf_variants and the engine use
(full residency, lazily allocated second slot, small warm-up launch first).  Prints per collect the device's
walked groups vs the submission.  Usage (GPU box): python tools/debug/epilogue_diag.py"""
import ctypes as C
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import torch  # noqa: E402,F401
from keyhuntm1cpu_amd import khhost  # noqa: E402
from keyhuntm1cpu_amd.khbsgs import Engine, Cand, Degenerate, Stats  # noqa: E402

t = khhost.Tables(None, 1, threads=16)
bf, nb, bits, h = t.bloom_concat(1)
gsn = t.giant_table()
offs, gpl = t.lane_offsets()
tgt = khhost.pubkey(0x2832ED74F2B5E35EE)
jobs = int(os.environ.get("JOBS", "4096"))
centres = b"".join(t.chunk_centre((1 << 65) + c * (1 << 45), tgt) for c in range(jobs))
gate, glog = t.gate()


def raw_collect(e):
    cand = (Cand * 4096)()
    deg = (Degenerate * 4096)()
    st = Stats()
    rc = e.L.khb_collect(e.h, cand, 4096, deg, 4096, C.byref(st))
    return rc, st


def run(label, reserve, warm, n_launch, gjobs, groups):
    e = Engine(0)
    e.load_bloom(bf, nb, bits, h)
    e.load_gate(gate, glog, t.gate_probes())
    e.load_giant_table(gsn)
    e.load_lane_offsets(offs, gpl)
    if reserve:
        e.reserve_slots(2)
    if warm:
        e.scan(centres[:64 * 8], 0, 64)
    c = centres[:64 * gjobs]
    exp = gjobs * groups * 1024
    e.submit(c, 0, groups)
    res = []
    for i in range(n_launch - 1):
        e.submit(c, 0, groups)
        rc, st = raw_collect(e)
        res.append((rc, st.giant_steps, exp, round(st.kernel_ms, 2), round(st.shader_mhz, 1)))
    rc, st = raw_collect(e)
    res.append((rc, st.giant_steps, exp, round(st.kernel_ms, 2), round(st.shader_mhz, 1)))
    e.close()
    bad = [r for r in res if r[0] or r[1] != r[2]]
    print(f"{label}: {'OK' if not bad else 'BAD'} {res}", flush=True)


run("small-jobs lazy slot1 warm", False, True, 4, 64, 4096)
run("full lazy slot1 no-warm", False, False, 4, jobs, 4096)
run("full reserved warm", True, True, 4, jobs, 4096)
run("full lazy slot1 warm", False, True, 4, jobs, 4096)
