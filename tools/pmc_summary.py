"""Summarise rocprofv3 outputs of tools/profile_bench.sh for k_giant_scan.
Usage: python tools/pmc_summary.py gpurun_out/<tag> [--write-latest]
Writes profiles/pmc_latest.json with --write-latest (read by bench.py for roofline.traffic)."""
import csv
import json
import os
import statistics
import sys
from collections import defaultdict

d = sys.argv[1]
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_dispatch(path, counter):
    agg = defaultdict(float)
    for r in csv.DictReader(open(path)):
        if "k_giant_scan" in r["Kernel_Name"] and r["Counter_Name"] == counter:
            agg[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    return agg


fetch = per_dispatch(os.path.join(d, "fetch", "fetch_counter_collection.csv"), "FETCH_SIZE")
write = per_dispatch(os.path.join(d, "write", "write_counter_collection.csv"), "WRITE_SIZE")
bench = json.load(open(os.path.join(d, "bench.json")))
chunks = bench["config"]["chunks_per_step"]
steps_per_launch = bench["config"]["giant_steps_per_step"]
# the largest dispatches are the full-size launches (warmup + timed); small ones are partial
fmax = max(fetch.values())
f_full = [v for v in fetch.values() if v > 0.9 * fmax]
w_full = sorted(write.values())[-len(f_full):]
f_kib, w_kib = statistics.mean(f_full), statistics.mean(w_full)
valu_path = os.path.join(d, "valu", "valu_counter_collection.csv")
valu = {}
if os.path.exists(valu_path):
    for cn in ("SQ_INSTS_VALU", "VALUBusy", "OccupancyPercent"):
        v = per_dispatch(valu_path, cn)
        vmax = max(v.values()) if v else 0
        full = [x for x in v.values() if x > 0.9 * vmax] if cn == "SQ_INSTS_VALU" else list(v.values())
        valu[cn] = statistics.mean(full) if full else None
stats = list(csv.DictReader(open(os.path.join(d, "trace", "trace_kernel_stats.csv"))))
scan = [r for r in stats if "k_giant_scan" in r["Name"]]
out = {
    "kernel": "k_giant_scan",
    "k": int(bench["config"]["workload"].split("-k ")[1].split()[0]),
    "chunks_per_launch": chunks,
    "giant_steps_per_launch": steps_per_launch,
    "dispatches_averaged": len(f_full),
    "fetch_size_kib": f_kib,
    "write_size_kib": w_kib,
    "hbm_bytes_per_launch": int((f_kib + w_kib) * 1024),
    "bytes_per_giant_step": round((f_kib + w_kib) * 1024 / steps_per_launch, 2),
    "trace_avg_ns": float(scan[0]["AverageNs"]) if scan else None,
    "valu_instr_per_giant_step": round(valu["SQ_INSTS_VALU"] * 64 / steps_per_launch, 1) if valu.get("SQ_INSTS_VALU") else None,
    "valu_busy_pct": round(valu["VALUBusy"], 2) if valu.get("VALUBusy") else None,
    "occupancy_pct": round(valu["OccupancyPercent"], 2) if valu.get("OccupancyPercent") else None,
    "valu_source": os.path.relpath(valu_path, REPO) if valu else None,
    "note": "FETCH_SIZE+WRITE_SIZE (KiB) x 1024 per full-size dispatch, uncorrected: the access mix "
            "(1-B random bloom probes, 16-B scratch streams, LDS-free spills) has no gfx950 calibration, and "
            "FETCH_SIZE counts Infinity-Cache hits (MI355X_MICROARCH.md HBM section)",
    "source": os.path.relpath(d, REPO),
}
print(json.dumps(out, indent=1))
if "--write-latest" in sys.argv:
    json.dump(out, open(os.path.join(REPO, "profiles", "pmc_latest.json"), "w"), indent=1)
