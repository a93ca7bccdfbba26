"""profiles/pmc_latest.json from the PMC passes of tools/gpu/round_profile.sh (bench.py reads it for
roofline.traffic and the executed VALU figures).

Inputs (rocprofv3 --pmc CSVs, one timed k_giant_scan launch each, JOBS chunks of the default k=1
geometry; the tiny first dispatch of perf_variants is skipped):
  pmc_fetch_0   FETCH_SIZE, TCC_EA0_RDREQ_sum with the real 2^28-bit gate
  pmc_fetch_13  the same launches plus the all-zero 1 KiB gate's (no gate traffic)
  pmc_write_0   WRITE_SIZE, TCC_EA0_WRREQ_sum
  pmc_sq        SQ_INSTS_VALU, SQ_ACTIVE_INST_VALU, GRBM_GUI_ACTIVE, ...
  pmc_sq2       (round 5, optional) SQ_INSTS_VALU, SQ_ACTIVE_INST_VALU, SQ_ACTIVE_INST_VALU2, SQ_INSTS_VALU_INT32/64,
                SQ_BUSY_CYCLES, SQ_WAVE_CYCLES, GRBM_GUI_ACTIVE: the VALU utilisation below
Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE counts half of a wide coalesced
streaming read, so the prefix stream's read bytes are 2 x the zero-gate launch's FETCH_SIZE;
WRITE_SIZE is exact for the 16-B-per-lane prefix stores.  The gate's reads are the extra memory-side
read requests of the real-gate launch (TCC_EA0_RDREQ real - zero) x 64 B (FETCH_SIZE = RDREQ x 64 B;
the scattered 8-B probe's request width is not calibrated, and Infinity-Cache hits are counted with
HBM reads: these are memory-side bytes, HBM or MALL).
VALU utilisation: a SIMD issues one VALU wave-instruction per quad-cycle, or two from different
waves when both are dual-issuable (SQ_ACTIVE_INST_VALU2 counts those quad-cycles).  SQ_ACTIVE_INST_VALU counts one
quad-cycle per VALU instruction (it equals SQ_INSTS_VALU here), so the quad-cycles in which the SIMD issued VALU
work are ACTIVE_INST_VALU - ACTIVE_INST_VALU2, and
  valu_util_pct = (ACTIVE_INST_VALU - ACTIVE_INST_VALU2) / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs / 4)
is the share of the launch's SIMD quad-cycles that issued VALU work (<= 100 % by construction).  The 4-cycle model
(rocprof's VALUBusy, ACTIVE_INST_VALU x 4 / SIMDs / per-XCD GRBM_GUI_ACTIVE) counts a dual-issued pair twice and
reads above 100 % (valu_busy_pct, kept for comparison).
The kernel configuration the record applies to (bench.py pmc_mismatch) is read from the profiled dispatch
itself: lanes = its grid size, waves per SIMD = lanes / (256 CUs x 4 SIMDs x 64), the level-0 gate from the kernel's
mode (k_giant_scan<7|8|9> are the gated scans), and the build (half prefix stream, groups per item, variant) from the
profiled library's khb_build_info (KHB_PMC_LIB, default the in-tree libkhbsgs.so).  A dispatch without those columns
is an error, not a default.
Usage: python tools/pmc_summary.py <dir with the pmc_* subdirs> <chunks per launch> [out.json] [k]
(k = 4: profiles/pmc_latest_k4.json, the record bench.py attaches to --k 4 lines)"""
import collections
import csv
import json
import os
import re
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
GROUPS = 4096          # k=1 default geometry: groups per chunk (cycles)
GROUPS_BY_K = {1: 4096, 4: 1024}   # cycles per chunk of the default -n 2^44 geometry
CUS, SIMDS = 256, 4
GATED_MODES = (7, 8, 9)   # scan_kernels.hpp kScanG, kScanG1, kScanG2


def dispatches(d, meta=False):
    out = collections.defaultdict(dict)
    info = {}
    with open(os.path.join(d, "pmc_counter_collection.csv"), newline="") as f:
        for r in csv.DictReader(f):
            if "k_giant_scan" in r["Kernel_Name"]:
                k = int(r["Dispatch_Id"])
                out[k][r["Counter_Name"]] = float(r["Counter_Value"])
                m = re.search(r"k_giant_scan<(\d+)>", r["Kernel_Name"])
                if not m or not r.get("Grid_Size"):
                    raise SystemExit(f"{d}: dispatch {k} has no kernel mode / grid size column")
                info[k] = {"mode": int(m.group(1)), "grid": int(r["Grid_Size"]),
                           "workgroup": int(r["Workgroup_Size"])}
    ks = sorted(out)
    return ([out[k] for k in ks], [info[k] for k in ks]) if meta else [out[k] for k in ks]


def kernel_config(meta: dict) -> dict:
    """lanes, waves per SIMD and gate of the profiled dispatch, and the profiled library's build words."""
    from keyhuntm1cpu_amd import khbsgs
    lanes = meta["grid"]
    b = khbsgs.build_info(os.environ.get("KHB_PMC_LIB") or None)
    return {"lanes": lanes, "waves_per_simd": lanes // (CUS * SIMDS * 64), "level0_gate": meta["mode"] in GATED_MODES,
            "kernel_mode": meta["mode"],
            "kernel_build": {k: b.get(k) for k in ("variant", "half_stream", "batch", "waves_per_simd", "gate1", "gate0")}}


def main():
    src, chunks = sys.argv[1], int(sys.argv[2])
    dst = sys.argv[3] if len(sys.argv) > 3 else os.path.join(REPO, "profiles", "pmc_latest.json")
    kk = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    steps = chunks * GROUPS_BY_K[kk] * 1024
    real_all, real_meta = dispatches(os.path.join(src, "pmc_fetch_0"), meta=True)
    real_f = real_all[-1]
    cfg = kernel_config(real_meta[-1])
    stream_alg = 16 if cfg["kernel_build"].get("half_stream") == "1" else 32
    both_f = dispatches(os.path.join(src, "pmc_fetch_13"))
    zero_f = both_f[-1]                    # the zero gate runs after the real one in perf_variants
    real_w = dispatches(os.path.join(src, "pmc_write_0"))[-1]
    sq = dispatches(os.path.join(src, "pmc_sq"))[-1]
    stream_rd = 2 * zero_f["FETCH_SIZE"] * 1024
    stream_wr = real_w["WRITE_SIZE"] * 1024
    gate_rd = (real_f["TCC_EA0_RDREQ_sum"] - zero_f["TCC_EA0_RDREQ_sum"]) * 64
    xcds = 8
    out = {
        "kernel": "k_giant_scan", "k": kk, **cfg,
        "chunks_per_launch": chunks, "giant_steps_per_launch": steps,
        "fetch_size_kib_real_gate": real_f["FETCH_SIZE"], "fetch_size_kib_zero_gate": zero_f["FETCH_SIZE"],
        "write_size_kib": real_w["WRITE_SIZE"],
        "ea_rdreq_real_gate": real_f["TCC_EA0_RDREQ_sum"], "ea_rdreq_zero_gate": zero_f["TCC_EA0_RDREQ_sum"],
        "ea_wrreq": real_w["TCC_EA0_WRREQ_sum"],
        "prefix_stream_read_bytes_per_giant_step": round(stream_rd / steps, 2),
        "prefix_stream_write_bytes_per_giant_step": round(stream_wr / steps, 2),
        "gate_read_requests_per_giant_step": round(gate_rd / 64 / steps, 4),
        "gate_read_bytes_per_giant_step": round(gate_rd / steps, 2),
        "hbm_bytes_per_launch": int(stream_rd + stream_wr + gate_rd),
        "bytes_per_giant_step": round((stream_rd + stream_wr + gate_rd) / steps, 2),
        "algorithmic_bytes_per_giant_step": stream_alg + 8,
        "valu_instr_per_giant_step": round(sq["SQ_INSTS_VALU"] * 64 / steps, 1),
        "valu_busy_pct": round(100 * sq["SQ_ACTIVE_INST_VALU"] * 4 / 1024 / (sq["GRBM_GUI_ACTIVE"] / xcds), 2),
        "valu_source": os.path.relpath(os.path.join(src, "pmc_sq"), REPO),
        "note": "traffic = prefix-stream reads (2 x FETCH_SIZE of the zero-gate launch, the gfx950 streaming-read "
                "correction) + prefix-stream writes (WRITE_SIZE) + the gate's extra memory-side read requests x 64 B; "
                "algorithmic = the prefix stream written and read once (16 + 16 B per giant step; 8 + 8 B with the "
                "half prefix stream, which stores every second prefix) + one 8-B gate probe per giant step. "
                "The gate's lines are fetched whole (64 B per 8-B probe); the counters do not separate "
                "Infinity-Cache hits from HBM. VALUBusy = ACTIVE_INST_VALU x 4 / 1024 SIMDs / (GRBM_GUI_ACTIVE / 8 XCDs).",
        "source": os.path.relpath(src, REPO),
    }
    sq2_dir = os.path.join(src, "pmc_sq2")
    if os.path.isdir(sq2_dir):
        q = dispatches(sq2_dir)[-1]
        quads = 1024 * q["GRBM_GUI_ACTIVE"] / xcds / 4
        out.update({
            "valu_util_pct": round(100 * (q["SQ_ACTIVE_INST_VALU"] - q["SQ_ACTIVE_INST_VALU2"]) / quads, 2),
            "valu_dual_issue_frac": round(2 * q["SQ_ACTIVE_INST_VALU2"] / q["SQ_INSTS_VALU"], 4),
            "valu_int32_frac": round(q["SQ_INSTS_VALU_INT32"] / q["SQ_INSTS_VALU"], 4),
            "valu_int64_frac": round(q["SQ_INSTS_VALU_INT64"] / q["SQ_INSTS_VALU"], 4),
            "valu_util_basis": "(SQ_ACTIVE_INST_VALU - SQ_ACTIVE_INST_VALU2) / SIMD quad-cycles (1024 SIMDs x "
                               "GRBM_GUI_ACTIVE / 8 XCDs / 4): the share of quad-cycles issuing VALU work, dual-issued "
                               "pairs counted once",
            "valu_util_source": os.path.relpath(sq2_dir, REPO)})
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
