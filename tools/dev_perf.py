"""Developer perf probe (not the bench): k=1 default geometry tables from the oracle, then time
the scan kernel for a few launch shapes.  Usage: python tools/dev_perf.py [gpl ...]"""
import sys
import time

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from oracle import ora  # noqa: E402
from keyhuntm1cpu_amd.khbsgs import Engine  # noqa: E402

t0 = time.time()
bs = ora.Bsgs(None, 1, 16)
print(f"tables {time.time()-t0:.1f}s m={bs.m} cycles={bs.cycles}", flush=True)
bf, nb, bits, h = bs.bloom_concat(1)
gsn = bs.giant_table()
key = 0x2832ED74F2B5E35EE
target = ora.pubkey(key)
base0 = 1 << 65
two_n = 2 * (1 << 44)
njobs = int(sys.argv[1]) if len(sys.argv) > 1 else 128
centres = b"".join(bs.chunk_start(base0 + c * two_n, target).be64() for c in range(njobs))
for gpl in [int(x) for x in sys.argv[2:]] or [4, 8]:
    n_off = (bs.cycles + gpl - 1) // gpl
    offs = [bytes(64)] + [ora.negation(ora.pubkey(m * gpl * 2048 * bs.m)).be64() for m in range(1, n_off)]
    for lanes in (65536, 131072):
        with Engine(0, lanes=lanes) as e:
            e.load_bloom(bf, nb, bits, h)
            e.load_giant_table(gsn)
            e.load_lane_offsets(b"".join(offs), gpl)
            e.scan(centres[: 64 * 8], 0, 64)  # warm-up
            for rep in range(2):
                t = time.time()
                cands, deg, st = e.scan(centres, 0, bs.cycles)
                wall = time.time() - t
                print(f"gpl={gpl} lanes={lanes} jobs={njobs} steps={st.giant_steps:.3e} kernel={st.kernel_ms:.1f}ms "
                      f"wall={wall*1e3:.1f}ms rate={st.giant_steps/st.kernel_ms/1e6:.3f} G/s cands={st.n_cand}",
                      flush=True)
