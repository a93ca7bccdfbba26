"""Device-busy time per step of a kernel from a rocprofv3 --kernel-trace CSV (bench.py's roofline basis).

Two submission slots keep two k_giant_scan launches in flight, so a launch's span
overlaps its neighbours' and the average launch duration exceeds the wall time per step.  The busy
time is the union of the launch intervals: over the last `--steps` launches of the kernel (the timed
steps follow the warmup ones), union / steps is directly comparable with bench.py's
roofline.kernel_busy_ms_per_step (the same union, from HIP events) and must not exceed ms_per_step.

Usage: python tools/trace_union.py <kernel_trace.csv> --kernel k_giant_scan --steps K [--bench bench.json]
Prints one JSON object: launches used, average launch ms, union ms per step, and (with --bench) the
line's kernel_busy_ms_per_step, ms_per_step and their ratio.
"""
from __future__ import annotations

import argparse
import csv
import json


def intervals(path: str, kernel: str) -> list[tuple[int, int]]:
    out = []
    with open(path, newline="") as f:
        for row in csv.DictReader(f):
            if kernel in row["Kernel_Name"]:
                out.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"])))
    out.sort()
    return out


def union_ns(iv: list[tuple[int, int]]) -> int:
    tot, b, e = 0, 0, -1
    for s, t in sorted(iv):
        if s > e:
            tot += max(0, e - b)
            b, e = s, t
        else:
            e = max(e, t)
    return tot + max(0, e - b)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--kernel", default="k_giant_scan")
    ap.add_argument("--steps", type=int, required=True, help="timed launches (the last ones in the trace)")
    ap.add_argument("--bench", help="the bench.py JSON line of the same command")
    a = ap.parse_args()
    iv = intervals(a.trace, a.kernel)
    if len(iv) < a.steps:
        raise SystemExit(f"{len(iv)} launches of {a.kernel} in the trace, {a.steps} requested")
    timed = iv[-a.steps:]
    out = {"trace": a.trace, "kernel": a.kernel, "launches_in_trace": len(iv), "launches_used": len(timed),
           "launch_ms_avg": round(sum(t - s for s, t in timed) / len(timed) / 1e6, 3),
           "busy_ms_per_step": round(union_ns(timed) / len(timed) / 1e6, 3),
           "span_ms_per_step": round((timed[-1][1] - timed[0][0]) / len(timed) / 1e6, 3)}
    if a.bench:
        with open(a.bench) as f:
            line = json.loads([ln for ln in f if ln.startswith("{")][-1])
        b = line["roofline"].get("kernel_busy_ms_per_step")
        out.update({"bench_kernel_busy_ms_per_step": b, "bench_ms_per_step": line["ms_per_step"],
                    "bench_kernel_ms_avg": line["roofline"].get("kernel_ms_avg"),
                    "bench_kernel_event_ms_avg": line["roofline"].get("kernel_event_ms_avg")})
        if b:
            out["trace_over_bench_busy"] = round(out["busy_ms_per_step"] / b, 4)
        if out["bench_kernel_event_ms_avg"]:     # rocprof's per-launch duration against the bench's events
            out["trace_over_bench_launch"] = round(out["launch_ms_avg"] / out["bench_kernel_event_ms_avg"], 4)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
