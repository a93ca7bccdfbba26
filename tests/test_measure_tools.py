"""CPU: the measurement tools behind bench.py's roofline.

tools/trace_union.py turns a rocprofv3 kernel trace into device-busy time per step (the union of
overlapping launch intervals, which bench.py computes from HIP events); tools/pmc_summary.py turns the
real-gate / zero-gate PMC passes into profiles/pmc_latest.json's corrected traffic.  Both are checked
on synthetic inputs with known answers, and the committed pmc_latest.json against its own raw CSVs.
"""
from __future__ import annotations

import csv
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))

import pmc_summary  # noqa: E402
import trace_union  # noqa: E402


def test_union_of_overlapping_launches():
    # two slots: each launch overlaps the next; gaps are not busy time
    iv = [(0, 10), (8, 20), (18, 30), (40, 50), (45, 47)]
    assert trace_union.union_ns(iv) == 30 + 10
    assert trace_union.union_ns([]) == 0
    assert trace_union.union_ns([(5, 5)]) == 0
    assert trace_union.union_ns([(0, 4), (4, 9)]) == 9


def _trace(path, rows):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        for name, s, e in rows:
            w.writerow({"Kernel_Name": name, "Start_Timestamp": s, "End_Timestamp": e})


def test_trace_union_cli_uses_the_last_launches(tmp_path):
    # 2 warmup + 3 timed launches of k_giant_scan (ms in ns), plus another kernel that must be ignored
    ms = 1_000_000
    rows = [("void khbk::k_giant_scan<7>(khbk::ScanArgs)", s * ms, e * ms)
            for s, e in ((0, 100), (90, 190), (180, 280), (270, 370), (360, 460))]
    rows.append(("k_expand_offsets", 0, 10 * ms))
    tr = tmp_path / "trace.csv"
    _trace(tr, rows)
    bench = tmp_path / "bench.json"
    bench.write_text(json.dumps({"ms_per_step": 93.5, "roofline": {"kernel_busy_ms_per_step": 93.3,
                                                                   "kernel_ms_avg": 100.0}}) + "\n")
    out = subprocess.run([sys.executable, os.path.join(REPO, "tools", "trace_union.py"), str(tr), "--steps", "3",
                          "--bench", str(bench)], capture_output=True, text=True, check=True)
    d = json.loads(out.stdout)
    assert d["launches_in_trace"] == 5 and d["launches_used"] == 3
    assert d["launch_ms_avg"] == 100.0
    assert d["busy_ms_per_step"] == round((460 - 180) / 3, 3)      # union of [180,280]+[270,370]+[360,460]
    assert d["trace_over_bench_busy"] == round(d["busy_ms_per_step"] / 93.3, 4)


def _pmc(d, dispatches):
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "pmc_counter_collection.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Grid_Size", "Kernel_Name", "Workgroup_Size", "Counter_Name",
                                          "Counter_Value"])
        w.writeheader()
        for did, counters in dispatches:
            for k, v in counters.items():
                w.writerow({"Dispatch_Id": did, "Grid_Size": 262144, "Workgroup_Size": 256,
                            "Kernel_Name": "void khbk::k_giant_scan<8>(khbk::ScanArgs)", "Counter_Name": k,
                            "Counter_Value": v})


def test_pmc_summary_corrections(tmp_path):
    chunks = 2
    steps = chunks * 4096 * 1024
    # zero gate: the prefix stream only (16 B read per step, counted at half by FETCH_SIZE; 16 B
    # written); real gate: + one 64-B request per step
    rd_zero = steps * 16 / 128                 # 128-B requests, tallied as 64 B each
    fetch_zero_kib = rd_zero * 64 / 1024
    rd_real = rd_zero + steps
    _pmc(tmp_path / "pmc_fetch_0", [(4, {"FETCH_SIZE": 1.0, "TCC_EA0_RDREQ_sum": 16.0}),
                                    (7, {"FETCH_SIZE": rd_real * 64 / 1024, "TCC_EA0_RDREQ_sum": rd_real})])
    _pmc(tmp_path / "pmc_fetch_13", [(4, {"FETCH_SIZE": 1.0, "TCC_EA0_RDREQ_sum": 16.0}),
                                     (7, {"FETCH_SIZE": rd_real * 64 / 1024, "TCC_EA0_RDREQ_sum": rd_real}),
                                     (9, {"FETCH_SIZE": fetch_zero_kib, "TCC_EA0_RDREQ_sum": rd_zero})])
    _pmc(tmp_path / "pmc_write_0", [(7, {"WRITE_SIZE": steps * 16 / 1024, "TCC_EA0_WRREQ_sum": steps / 4})])
    _pmc(tmp_path / "pmc_sq", [(7, {"SQ_INSTS_VALU": steps * 700 / 64, "SQ_ACTIVE_INST_VALU": steps * 700 / 64,
                                    "GRBM_GUI_ACTIVE": 8.0 * steps * 700 / 64 * 4 / 1024})])
    out = tmp_path / "pmc.json"
    subprocess.run([sys.executable, os.path.join(REPO, "tools", "pmc_summary.py"), str(tmp_path), str(chunks),
                    str(out)], capture_output=True, text=True, check=True)
    d = json.loads(out.read_text())
    assert d["prefix_stream_read_bytes_per_giant_step"] == 16.0
    assert d["prefix_stream_write_bytes_per_giant_step"] == 16.0
    assert d["gate_read_requests_per_giant_step"] == 1.0
    assert d["bytes_per_giant_step"] == 96.0
    assert d["hbm_bytes_per_launch"] == 96 * steps
    assert d["valu_instr_per_giant_step"] == 700.0
    assert d["valu_busy_pct"] == 100.0
    # the configuration comes from the dispatch (grid 262,144 lanes, k_giant_scan<8> = kScanG1) and the library
    assert (d["lanes"], d["waves_per_simd"], d["level0_gate"], d["kernel_mode"]) == (262144, 4, True, 8)
    assert d["kernel_build"]["variant"] == "product"
    assert d["algorithmic_bytes_per_giant_step"] == (24 if d["kernel_build"]["half_stream"] == "1" else 40)


def test_pmc_summary_refuses_a_dispatch_without_its_configuration(tmp_path):
    """a PMC CSV whose k_giant_scan rows lack the grid size is an error, not a default."""
    d = tmp_path / "pmc_fetch_0"
    os.makedirs(d)
    with open(d / "pmc_counter_collection.csv", "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        w.writerow({"Dispatch_Id": 1, "Kernel_Name": "void khbk::k_giant_scan<8>(khbk::ScanArgs)",
                    "Counter_Name": "FETCH_SIZE", "Counter_Value": 1.0})
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "pmc_summary.py"), str(tmp_path), "1",
                        str(tmp_path / "o.json")], capture_output=True, text=True)
    assert r.returncode != 0 and "grid size" in (r.stderr + r.stdout)


@pytest.mark.parametrize("name", ["pmc_latest.json", "pmc_latest_k4.json"])
def test_committed_pmc_latest_reproduces_from_its_csvs(tmp_path, name):
    """profiles/pmc_latest.json (bench.py's roofline.traffic for k = 1) and pmc_latest_k4.json (for --k 4) equal a
    rerun of the summary on the raw CSVs they name."""
    with open(os.path.join(REPO, "profiles", name)) as f:
        cur = json.load(f)
    out = tmp_path / "again.json"
    subprocess.run([sys.executable, os.path.join(REPO, "tools", "pmc_summary.py"), os.path.join(REPO, cur["source"]),
                    str(cur["chunks_per_launch"]), str(out), str(cur["k"])], capture_output=True, text=True,
                   check=True)
    again = json.loads(out.read_text())
    for k in ("hbm_bytes_per_launch", "bytes_per_giant_step", "gate_read_requests_per_giant_step",
              "valu_instr_per_giant_step", "valu_util_pct", "valu_dual_issue_frac", "level0_gate", "lanes",
              "waves_per_simd"):
        assert again[k] == cur[k], k
    assert pmc_summary.GROUPS == 4096


def test_bench_traffic_matches_default_batch():
    """The committed PMC launch has the bench's auto batch at 4 waves/SIMD (8 work items per lane of 262,144
    lanes: 4,096 chunks of the k=1 geometry), so the default line's roofline.traffic is the measured launch;
    another --chunks scales the measured bytes per giant step and says so."""
    sys.path.insert(0, REPO)
    import bench
    with open(os.path.join(REPO, "profiles", "pmc_latest.json")) as f:
        pmc = json.load(f)
    lanes, per_item, cycles = 4 * 4 * 64 * 256, 8, 4096
    auto = 8 * (-(-lanes * per_item // cycles))
    assert pmc["k"] == 1 and pmc["chunks_per_launch"] == auto == 4096
    steps = auto * cycles * 1024
    assert bench.pmc_traffic(pmc, auto, steps) == {"traffic": pmc["hbm_bytes_per_launch"]}
    half = bench.pmc_traffic(pmc, auto // 2, steps // 2)
    assert abs(half["traffic"] - pmc["hbm_bytes_per_launch"] / 2) < 1e-3 * pmc["hbm_bytes_per_launch"]
    assert "scaled to 2048" in half["traffic_note"]


def test_pmc_summary_valu_utilisation(tmp_path):
    """The round-5 VALU utilisation: quad-cycles that issued VALU work (dual-issued pairs counted once) over
    the SIMD quad-cycles of the launch; 900 instructions with 100 dual-issued pairs in 1000 quad-cycles per
    SIMD -> 80 %, while the 4-cycle model reads 90 %."""
    chunks = 1
    steps = chunks * 4096 * 1024
    quads_per_simd = 1000.0
    insts = 900.0 * 1024
    base = {"FETCH_SIZE": 1.0, "TCC_EA0_RDREQ_sum": 1.0}
    _pmc(tmp_path / "pmc_fetch_0", [(1, base)])
    _pmc(tmp_path / "pmc_fetch_13", [(1, base), (2, base)])
    _pmc(tmp_path / "pmc_write_0", [(1, {"WRITE_SIZE": 1.0, "TCC_EA0_WRREQ_sum": 1.0})])
    grbm = 8 * quads_per_simd * 4
    _pmc(tmp_path / "pmc_sq", [(1, {"SQ_INSTS_VALU": insts, "SQ_ACTIVE_INST_VALU": insts, "GRBM_GUI_ACTIVE": grbm})])
    _pmc(tmp_path / "pmc_sq2", [(1, {"SQ_INSTS_VALU": insts, "SQ_ACTIVE_INST_VALU": insts,
                                     "SQ_ACTIVE_INST_VALU2": 100.0 * 1024, "SQ_INSTS_VALU_INT32": insts / 2,
                                     "SQ_INSTS_VALU_INT64": insts / 4, "GRBM_GUI_ACTIVE": grbm})])
    out = tmp_path / "pmc.json"
    subprocess.run([sys.executable, os.path.join(REPO, "tools", "pmc_summary.py"), str(tmp_path), str(chunks),
                    str(out)], capture_output=True, text=True, check=True)
    d = json.loads(out.read_text())
    assert d["valu_busy_pct"] == 90.0
    assert d["valu_util_pct"] == 80.0
    assert d["valu_dual_issue_frac"] == round(200 / 900, 4)
    assert d["valu_int32_frac"] == 0.5 and d["valu_int64_frac"] == 0.25
    assert steps


def test_power_summary_synthetic():
    """keyhuntm1cpu_amd/power.py's summary on synthetic samples (no amdsmi): averages, the cap fraction, energy
    per 1e9 units from the energy counter, the throttle-residency fractions; a disabled sampler reports why."""
    sys.path.insert(0, REPO)
    from keyhuntm1cpu_amd.power import PowerSampler
    ps = PowerSampler.disabled("test")
    assert ps.summary() == {"available": False, "error": "test"}
    ps = PowerSampler.disabled("test")
    ps.err, ps.cap_w, ps.period = None, 1400.0, 0.05
    ps.samples = [{"t": float(i), "power_w": w, "gfxclk": [2100.0, 2200.0], "gfx_activity": 100.0,
                   "temp_hotspot": 50.0 + i, "temp_mem": 40.0, "throttle": "N/A", "indep_throttle": "N/A"}
                  for i, w in enumerate((1300.0, 1400.0, 1350.0))]
    ps._e0, ps._e1 = (0.0, 1000.0), (2.0, 3700.0)
    ps._r0 = {"ppt_residency_acc": 10.0, "socket_thm_residency_acc": 0.0, "vr_thm_residency_acc": 0.0,
              "hbm_thm_residency_acc": 0.0, "prochot_residency_acc": 0.0, "accumulation_counter": 100.0}
    ps._r1 = dict(ps._r0, ppt_residency_acc=90.0, accumulation_counter=200.0)
    s = ps.summary(work_units=27e9, seconds=2.0)
    assert s["power_w_avg"] == 1350.0 and s["gfxclk_mhz_avg"] == 2150.0
    assert s["power_w_from_energy"] == 1350.0 and s["energy_j"] == 2700.0
    assert s["at_cap_frac"] == round(1350 / 1400, 3)
    assert s["joules_per_1e9_giant_steps"] == 100.0
    assert s["ppt_residency_frac"] == 0.8 and s["prochot_residency_frac"] == 0.0
    assert "throttle_status_seen" not in s


def test_pmc_record_attaches_only_to_its_configuration():
    """bench.py attaches profiles/pmc_latest.json's traffic / VALU figures only to a run of the kernel configuration
    the record was measured on: the committed record matches the default k=1 gated 4-wave line, and a
    --no-gate, k=4 or other-lane-count run gets a note instead."""
    sys.path.insert(0, REPO)
    import bench
    with open(os.path.join(REPO, "profiles", "pmc_latest.json")) as f:
        pmc = json.load(f)
    default = {"k": 1, "level0_gate": True, "lanes": 262144, "waves_per_simd": 4}
    if "kernel_build" in pmc:
        default["kernel_build"] = pmc["kernel_build"]
    assert bench.pmc_mismatch(pmc, default) is None
    for change in ({"level0_gate": False}, {"k": 4}, {"lanes": 196608, "waves_per_simd": 3},
                   {"kernel_build": {"variant": "half", "half_stream": "0"}}):
        note = bench.pmc_mismatch(pmc, dict(default, **change))
        assert note and "not measured for this run" in note and all(k in note for k in change)
    assert bench.pmc_mismatch({"k": 1}, default)          # a record without its configuration never matches


def test_power_handle_matches_full_pci_address():
    """the amdsmi handle is matched on the full domain:bus:device, and a rank whose GPU is not found gets
    no power block instead of another GPU's figures."""
    sys.path.insert(0, REPO)
    from keyhuntm1cpu_amd.power import _handle_for_bdf

    class FakeSmi:
        bdfs = {"h0": "0000:8b:00.0", "h1": "0001:8b:00.0", "h2": "0000:8b:01.0"}

        def amdsmi_get_processor_handles(self):
            return list(self.bdfs)

        def amdsmi_get_gpu_device_bdf(self, h):
            return self.bdfs[h]
    smi = FakeSmi()
    assert _handle_for_bdf(smi, "0001:8b:00") == ("h1", None)       # same bus, other domain
    assert _handle_for_bdf(smi, "0000:8b:01") == ("h2", None)       # same bus, other device
    h, why = _handle_for_bdf(smi, "0000:9c:00")
    assert h is None and "0000:9c:00" in why
    h, why = _handle_for_bdf(smi, None)
    assert h is None and "3 amdsmi handles" in why
    FakeSmi.bdfs = {"h0": "0000:8b:00.0"}
    assert _handle_for_bdf(FakeSmi(), None) == ("h0", None)


def test_energy_split_reproduces_design():
    """tools/energy_split.py recomputes DESIGN.md §5's energy table from the committed evidence (r06c/d/f/g, r05c,
    pmc_latest.json): VALU 12.6 nJ, non-VALU <= 0.13, zero-memory build 13.5, memory side in situ 4.85, product 18.35
    nJ per giant step, and the product at 94.0 % of the compute-only ceiling."""
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "energy_split.py")], capture_output=True,
                       text=True, check=True)
    d = json.loads(r.stdout)
    assert abs(d["valu_nj"] - 12.6) < 0.05 and d["non_valu_nj_total"] < 0.135
    assert abs(d["zero_memory"]["nj"] - 13.5) < 0.05 and abs(d["memory_side_in_situ_nj"] - 4.85) < 0.01
    assert abs(d["product"]["nj"] - 18.35) < 0.01 and abs(d["product_over_compute_ceiling"] - 0.940) < 0.001
    assert abs(d["compute_predicted_nj"] - d["zero_memory"]["nj"]) < 1.0      # within 1 nJ
    assert d["icache_miss_frac"] < 1e-4
