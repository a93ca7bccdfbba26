"""A/B timing of libkhbsgs kernel variants in ONE process (interleaved rounds, median).
Usage: python tools/perf_variants.py [lib.so ...]   (default: the product library + lib/variants/*)
Tables: product host engine, default geometry (k=1, or K=...), puzzle #66 target, JOBS (256) chunks
per launch.
GATE=0|1|both (default both): run every library without / with the level-0 gate.
GATE_LOG2S=23,24 adds gates of those sizes, folded from the tables' gate (64-bit block i of a
2^(L-1)-bit map is block i | block i + 2^(L-7) of the 2^L map: the same map a 2^(L-1) build writes,
the block index being (x mod 2^32) mod 2^(L-6)).
GATE_ZERO=L adds an all-zero gate of 2^L bits (L >= 13): the same gate code and instructions, but every
block load hits the vector L1 (1 KiB at L = 13) and no x passes, which isolates the cost of the real
gate's cache misses (verdict r2 item 4); its candidate set is empty by construction."""
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
t = khhost.Tables(None, int(os.environ.get("K", "1")), threads=16)
bf, nb, bits, h = t.bloom_concat(1)
gsn = t.giant_table()
offs, gpl = t.lane_offsets()
tgt = khhost.pubkey(0x2832ED74F2B5E35EE)
jobs = int(os.environ.get("JOBS", "256"))
centres = b"".join(t.chunk_centre((1 << 65) + c * (1 << 45), tgt) for c in range(jobs))
gate, glog = t.gate()
gmode = os.environ.get("GATE", "both")
gsets = [0, glog] if gmode == "both" else [glog if gmode == "1" else 0]
gates = {glog: gate}
import numpy as np  # noqa: E402
for lg in [int(v) for v in os.environ.get("GATE_LOG2S", "").split(",") if v]:
    blocks = np.frombuffer(gate, np.uint64)
    gates[lg] = np.bitwise_or.reduce(blocks.reshape(1 << (glog - lg), -1), axis=0).tobytes()
    gsets.append(lg)
if int(os.environ.get("GATE_ZERO", "0") or 0):
    lz = int(os.environ["GATE_ZERO"])
    gates[-lz] = bytes((1 << lz) // 8)
    gsets.append(-lz)
# One Engine at a time: each owns ~35 GB of scratch per submission slot (262,144 lanes), so every (variant, gate) pair
# gets its own context per round, opened, timed and closed before the next one (round 3 kept all of them
# open at once and ran out of HBM with six variants, gpurun_out/r03m/ab.txt).
# STAGE1=default,0,22: time every real gate with the library's default stage-1 fold (KHB_GATE_STAGE1_AUTO),
# with none (0), and with a fold of 2^22 bytes (khb_set_gate_stage1)
stage1s = [v for v in os.environ.get("STAGE1", "default").split(",") if v]
configs = [(p, (g, s1)) for p in paths for g in gsets for s1 in (stage1s if g > 0 else ["default"])]


def cfg_name(p, gs):
    g, s1 = gs
    return (os.path.basename(p) + (f" +gate{g}" if g > 0 else f" +zerogate{-g}" if g else "")
            + ("" if s1 == "default" else " +no stage1" if s1 == "0" else f" +stage1 2^{s1}B"))


def open_engine(p, gs):
    g, s1 = gs
    e = Engine(0, lib_path=p)
    e.load_bloom(bf, nb, bits, h)
    if s1 != "default":
        e.set_gate_stage1(int(s1))
    if g:
        e.load_gate(gates[g], abs(g), t.gate_probes())
    e.load_giant_table(gsn)
    e.load_lane_offsets(offs, gpl)
    e.scan(centres[:64 * 8], 0, 64)               # warm: code object load, first-touch of the tables
    return e


# PIPE=n (n >= 2): time n back-to-back launches with two in flight, as the engine runs them, instead of one
# synchronous launch (whose ramp and tail the queue otherwise hides)
pipe = int(os.environ.get("PIPE", "0") or 0)
times = {cfg_name(p, gs): [] for p, gs in configs}
mhz = {n: [] for n in times}
watts = {n: [] for n in times}
# POWER=1: board power over each timed pipe (keyhuntm1cpu_amd/power.py; amdsmi, not HIP)
use_power = os.environ.get("POWER", "0") == "1"
if use_power:
    from keyhuntm1cpu_amd.power import PowerSampler
ncand = {}
ref = {}
for rnd in range(int(os.environ.get("ROUNDS", "3"))):
    for p, gs in configs:
        g = gs[0]
        n = cfg_name(p, gs)
        e = open_engine(p, gs)
        try:
            if rnd == 0:
                print(f"{n}: lanes {e.lanes()}", flush=True)
            if pipe:
                # PIPE=n: n launches with two in flight (the engine's queue depth), wall time per launch
                ps = PowerSampler(period=0.02) if use_power else None
                e.submit(centres, 0, t.cycles)
                if ps:
                    ps.__enter__()
                t0 = time.perf_counter()
                for _ in range(pipe - 1):
                    e.submit(centres, 0, t.cycles)
                    c, d, st = e.collect()
                c, d, st = e.collect()
                kms = 1e3 * (time.perf_counter() - t0) / pipe
                if ps:
                    ps.__exit__(None, None, None)
                    sm = ps.summary()
                    watts[n].append((sm.get("power_w_from_energy") or sm.get("power_w_avg") or 0.0,
                                     sm.get("ppt_residency_frac")))
            else:
                c, d, st = e.scan(centres, 0, t.cycles)
                kms = st.kernel_ms
        finally:
            e.close()
        times[n].append(kms)
        mhz[n].append(getattr(st, "shader_mhz", 0.0))
        ncand[n] = len(c)
        timing_only = [v for v in os.environ.get("TIMING_ONLY", "").split(",") if v]
        if "_p" in n.split()[0] or "nonop" in n or "_rm" in n or "_scr" in n or any(v in n for v in timing_only):
            continue                               # timing-only experiments: candidates not comparable
        s = sorted(c)
        if g < 0:                                  # the zero gate: nothing passes
            assert not s, f"{n}: a zero gate passed candidates"
            continue
        ref.setdefault(g, s)
        assert s == ref[g], f"{n}: candidate set differs"
for g in ref:   # a gate keeps a subset of the L1 candidates
    assert 0 not in ref or set(ref[g]) <= set(ref[0])
steps = jobs * t.cycles * 1024
for n in times:
    med = statistics.median(times[n])
    pw = ""
    if watts[n]:
        w = statistics.median(x[0] for x in watts[n])
        ppt = [x[1] for x in watts[n] if x[1] is not None]
        pw = (f"  {w:7.1f} W  {w * med * 1e-3 / (steps / 1e9):6.2f} J/1e9 steps"
              + (f"  ppt {statistics.median(ppt):.3f}" if ppt else ""))
    print(f"{n:48s} median {med:8.2f} ms  min {min(times[n]):8.2f}  {steps / med / 1e6:8.3f} G steps/s"
          f"  cand {ncand[n]}  clock {statistics.median(mhz[n]):7.1f} MHz{pw}", flush=True)
for n in times:
    print(f"  {n}: rounds (ms) {[round(x, 2) for x in times[n]]}", flush=True)
