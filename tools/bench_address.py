"""-m address throughput (BASELINE config E): keyhunt -m address -f tests/unsolvedpuzzles.rmd on one
MI355X, sequential chunks of -n keys from 2^70 (puzzle #71's range), reported as Mkeys/s with the
VALU roofline of the hash path.  Prints one JSON line.

Usage: python tools/bench_address.py [--search 2] [--chunks 24] [--n 0x100000000]
(24 chunks of 2^32 keys = three launches of eight work items per lane, two queued at a time.)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

# 32-bit VALU operations per key, counted from the algorithms (FIPS 180-4 / RIPEMD-160 as restated in
# device/hash160.hpp): a SHA-256 compression is 64 rounds x 22 + 48 schedule
# words x 13 = 2032, a RIPEMD-160 compression 160 steps x 9 = 1440; the EC walk is ~4.5 field
# multiplies per key (x and y) at ~150 VALU each.
SHA_BLOCK, RMD_BLOCK, EC_PER_KEY = 2032, 1440, 680
OPS = {0: 2 * SHA_BLOCK + RMD_BLOCK + EC_PER_KEY,            # uncompressed: 65-byte message, 2 blocks
       1: 2 * (SHA_BLOCK + RMD_BLOCK) + EC_PER_KEY - 150,    # compressed 02 + 03 from x (no y)
       2: 4 * SHA_BLOCK + 3 * RMD_BLOCK + EC_PER_KEY}
# Executed VALU lane-instructions per key, -l both (rocprofv3 --pmc SQ_INSTS_VALU x 64 / keys of one
# 8-chunk launch, profiles/r02w/addr_valu_counter_collection.csv: 4.968e12 wave-instr x 64 / 2^35 keys;
# VALUBusy 101.5 %: the kernel is at the VALU issue ceiling).
EXEC_PER_KEY = {2: 9253.4}
PEAK_T = 68.2   # measured v_add_u32 / v_xor issue, 111 lane-ops/clk/CU x 256 CU x 2.4 GHz (profiles/r01_intops2.txt)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--search", type=int, default=2, help="0 uncompress, 1 compress, 2 both (default, as keyhunt)")
    ap.add_argument("--chunks", type=int, default=24)
    ap.add_argument("--n", type=lambda s: int(s, 0), default=1 << 32)
    ap.add_argument("--warmup", type=int, default=1)
    args = ap.parse_args()
    import torch  # noqa: F401  (share torch's HIP runtime, as bench.py)
    from keyhuntm1cpu_amd import khhost
    with open(os.path.join(REPO, "tests", "golden", "address", "unsolvedpuzzles.rmd")) as f:
        text = f.read()
    t0 = time.time()
    A = khhost.Addr(text, n_seq=args.n, threads=16)
    t_build = time.time() - t0
    start = 1 << 70
    if args.warmup:
        A.search(start, start + args.warmup * args.n, search=args.search)
    t0 = time.time()
    found, st = A.search(start + args.warmup * args.n, start + (args.warmup + args.chunks) * args.n,
                         search=args.search)
    dt = time.time() - t0
    keys = st["keys"]
    rate = keys / dt
    kern = st["kernel_s"] / max(1, st["launches"])
    achieved = OPS[args.search] * keys / st["kernel_s"] / 1e12
    out = {
        "metric": "Mkeys/s (-m address, keys hashed and probed per second)",
        "value": round(rate / 1e6, 2),
        "unit": "Mkeys/s",
        "n_gpus": 1,
        "keys": keys,
        "seconds": round(dt, 3),
        "search": ["uncompress", "compress", "both"][args.search],
        "reference_keys_per_s": round(rate * (2 if args.search == 1 else 1) / 1e6, 2),
        "config": {"workload": "-m address -f tests/unsolvedpuzzles.rmd -b 71 (BASELINE configs[4])",
                   "targets": len(A.table()), "n_seq": hex(args.n), "chunks": st["chunks"],
                   "launches": st["launches"], "bloom_hits": st["hits"], "found": len(found),
                   "table_build_s": round(t_build, 2)},
        "roofline": {"bound": "valu", "unit": "Tops/s", "achieved": round(achieved, 3), "peak": PEAK_T,
                     "frac": round(achieved / PEAK_T, 4), "ops_per_key": OPS[args.search],
                     "achieved_wall": round(OPS[args.search] * rate / 1e12, 3),
                     "frac_wall": round(OPS[args.search] * rate / 1e12 / PEAK_T, 4),
                     "kernel": "k_giant_scan<address>", "kernel_ms_avg": round(kern * 1e3, 3)},
    }
    if args.search in EXEC_PER_KEY:
        e = EXEC_PER_KEY[args.search]
        out["roofline"]["executed"] = {
            "valu_lane_instr_per_key": e, "valu_busy_pct": 101.5,
            "valu_lane_instr_T_per_s_wall": round(e * rate / 1e12, 3),
            "pmc_source": "profiles/r02w/addr_valu_counter_collection.csv",
            "note": "fewer executed than algorithmic ops: v_bitop3 / v_alignbit / v_add3 fuse 2-3 simple ops"}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
