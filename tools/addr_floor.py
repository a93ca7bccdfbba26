"""One -m address launch per library (config E: tests/unsolvedpuzzles.rmd, -l both by default, 8 chunks of
2^32 keys from 2^70, the bench's launch) for PMC passes: rocprofv3 --pmc SQ_INSTS_VALU -- python3
tools/addr_floor.py <lib.so>.  With the product library the counter gives the executed VALU per key;
with the addrwalk build (tools/experiments/calib_build.sh addrwalk) it gives the x/y walk alone, the
walk term of the floor.  Prints one JSON line."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402,F401
from keyhuntm1cpu_amd import khhost  # noqa: E402
from keyhuntm1cpu_amd.khbsgs import Engine, LIB_PATH  # noqa: E402

lib_path = sys.argv[1] if len(sys.argv) > 1 else LIB_PATH
search = int(os.environ.get("SEARCH", "2"))
chunks = int(os.environ.get("CHUNKS", "8"))
n_seq = 1 << 32
with open(os.path.join(REPO, "tests", "golden", "address", "unsolvedpuzzles.rmd")) as f:
    A = khhost.Addr(f.read(), n_seq=n_seq, threads=16)
e = Engine(0, lib_path=lib_path)
bf, bits, h = A.bloom()
e.load_addr_bloom(bf, bits, h)
e.load_giant_table(A.giant_table())
offs, gpl = A.lane_offsets()
e.load_lane_offsets(offs, gpl)
groups = n_seq // 1024
base = 1 << 70
e.addr_scan(khhost.pubkey(base + 512), 0, 4096, search)            # warm
centres = b"".join(khhost.pubkey(base + c * n_seq + 512) for c in range(chunks))
t0 = time.perf_counter()
hits, st = e.addr_scan(centres, 0, groups, search)
dt = time.perf_counter() - t0
e.close()
keys = chunks * n_seq
print(json.dumps({"lib": os.path.basename(lib_path), "search": search, "keys": keys, "hits": len(hits),
                  "kernel_ms": round(st.kernel_ms, 2), "wall_s": round(dt, 3),
                  "mkeys_per_s": round(keys / (st.kernel_ms * 1e-3) / 1e6, 1),
                  "shader_mhz": round(getattr(st, "shader_mhz", 0.0), 1)}), flush=True)
