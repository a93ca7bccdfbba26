"""The energy per giant step by class recomputed from the committed evidence.

Inputs (all under profiles/):
  r06g/zero_mem.txt        perf_variants lines (two launches in flight, board power): the product with the real gate
                           and with the all-zero gate, and the zero-memory build (half stream folded into the caches)
                           with both; G steps/s and W per configuration
  r06c/valu_energy.jsonl   the "sleep" level (every wave resident, sleeping) and the SALU / SMEM / LDS prices
  r06d/valu_energy.jsonl   the L2-resident scratch (spill) price
  r06c/pmc_classes/        PMC instruction classes of one bench-sized product launch (SQ_INSTS_*)
  r06f/pmc_icache/         instruction fetches and I-cache misses of the same launch
  r05c/f64mul_time.jsonl   the field product's energy (fm_mul chains alone at full occupancy)
  pmc_latest.json          VALU lane-instructions per giant step of the product
Prints one JSON object; tests/test_measure_tools.py checks it against the figures DESIGN.md quotes.
Usage: python tools/energy_split.py"""
import collections
import csv
import json
import os
import re
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = os.path.join(REPO, "profiles")
STEPS = 4096 * 4096 * 1024          # giant steps of one bench-sized launch (the PMC launches)
VALU_PER_FM_MUL = 198               # VALU instructions of one fm_mul (ISA)


def jsonl(path):
    with open(path) as f:
        return [json.loads(l) for l in f if l.strip().startswith("{")]


def perf_lines(path):
    """{config: (G steps/s, W)} from perf_variants' summary lines."""
    out = {}
    pat = re.compile(r"^(\S+ \+\S+)\s+median .*?([\d.]+) G steps/s .*? ([\d.]+) W")
    with open(path) as f:
        for line in f:
            m = pat.match(line.strip())
            if m:
                out[m.group(1)] = (float(m.group(2)), float(m.group(3)))
    return out


def pmc_last(d):
    rows = collections.defaultdict(dict)
    with open(os.path.join(d, "pmc_counter_collection.csv"), newline="") as f:
        for r in csv.DictReader(f):
            if "k_giant_scan" in r["Kernel_Name"]:
                rows[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    return rows[max(rows)]


def main():
    e6c = {r["mode"]: r for r in jsonl(os.path.join(P, "r06c", "valu_energy.jsonl"))}
    e6d = {r["mode"]: r for r in jsonl(os.path.join(P, "r06d", "valu_energy.jsonl"))}
    sleep_w = statistics.mean(r["power_w"] for r in jsonl(os.path.join(P, "r06c", "valu_energy.jsonl"))
                              if r["mode"] == "sleep")
    runs = perf_lines(os.path.join(P, "r06g", "zero_mem.txt"))
    prod, prod_zero_gate = runs["libkhbsgs.so +gate28"], runs["libkhbsgs.so +zerogate13"]
    zmem_stream, zmem = runs["libkhbsgs_scr1half.so +gate28"], runs["libkhbsgs_scr1half.so +zerogate13"]
    nj = lambda gw: (gw[1] - sleep_w) / gw[0]            # nJ per giant step above sleep  # noqa: E731
    fm = [r for r in jsonl(os.path.join(P, "r05c", "f64mul_time.jsonl")) if r["kind"] == "u32"]
    fm_w = statistics.mean(r["power"]["power_w_from_energy"] for r in fm)
    fm_rate = statistics.mean(r["G_products_per_s"] for r in fm)
    pj_per_valu = (fm_w - sleep_w) / fm_rate / VALU_PER_FM_MUL * 1e3
    with open(os.path.join(P, "pmc_latest.json")) as f:
        valu = json.load(f)["valu_instr_per_giant_step"]
    cls = pmc_last(os.path.join(P, "r06c", "pmc_classes"))
    ic = pmc_last(os.path.join(P, "r06f", "pmc_icache"))
    per = lambda k: cls[k] / STEPS                        # wave-instructions per giant step  # noqa: E731
    vmem_lane = (cls["SQ_INSTS_VMEM_RD"] + cls["SQ_INSTS_VMEM_WR"]) * 64 / STEPS
    # known vector-memory lane-instructions per giant step: stream stores 0.5 + loads 0.5 + fold 1.0 + full gate 1.0
    scratch_lane = max(0.0, vmem_lane - 3.0)
    non_valu = {
        "salu": per("SQ_INSTS_SALU") * e6c["salu"]["pj_per_unit_above_sleep"] / 1e3,
        "smem": per("SQ_INSTS_SMEM") * e6c["smem"]["pj_per_unit_above_sleep"] / 1e3,
        "lds": per("SQ_INSTS_LDS") * 64 * e6c["lds"]["pj_per_unit_above_sleep"] / 1e3,
        "scratch_upper": scratch_lane * e6d["scratch_l2"]["pj_per_unit_above_sleep"] / 1e3,
    }
    out = {
        "sleep_w": round(sleep_w, 1),
        "pj_per_valu_instr": round(pj_per_valu, 2),
        "valu_instr_per_giant_step": valu,
        "valu_nj": round(valu * pj_per_valu / 1e3, 2),
        "non_valu_nj": {k: round(v, 4) for k, v in non_valu.items()},
        "non_valu_nj_total": round(sum(non_valu.values()), 3),
        "vmem_lane_instr_per_giant_step": round(vmem_lane, 3),
        "icache_miss_frac": round(ic["SQC_ICACHE_MISSES"] / ic["SQC_ICACHE_REQ"], 7),
        "ifetch_per_giant_step": round(ic["SQ_IFETCH"] / STEPS, 3),
        "product": {"g_steps_per_s": prod[0], "w": prod[1], "nj": round(nj(prod), 2)},
        "zero_gate": {"g_steps_per_s": prod_zero_gate[0], "w": prod_zero_gate[1], "nj": round(nj(prod_zero_gate), 2)},
        "cached_stream": {"g_steps_per_s": zmem_stream[0], "w": zmem_stream[1], "nj": round(nj(zmem_stream), 2)},
        "zero_memory": {"g_steps_per_s": zmem[0], "w": zmem[1], "nj": round(nj(zmem), 2)},
    }
    out["compute_predicted_nj"] = round(out["valu_nj"] + out["non_valu_nj_total"], 2)
    out["memory_side_in_situ_nj"] = round(out["product"]["nj"] - out["zero_memory"]["nj"], 2)
    out["gate_alone_nj"] = round(out["product"]["nj"] - out["zero_gate"]["nj"], 2)
    out["stream_alone_nj"] = round(out["product"]["nj"] - out["cached_stream"]["nj"], 2)
    out["product_over_compute_ceiling"] = round(prod[0] / zmem[0], 4)
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
