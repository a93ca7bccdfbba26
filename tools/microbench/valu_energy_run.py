"""Energy per instruction class (tools/microbench/valu_energy.hip) under board-power sampling: each mode runs as a
child process for SECONDS while this process (amdsmi only, no HIP) samples power; the `sleep` mode (every wave
resident, sleeping) is the baseline.  Prints one JSON line per mode with W, clock, the firmware's power-limit
residency and the dynamic energy above the baseline per unit (pJ per lane-instruction / byte / load).
Usage: python tools/microbench/valu_energy_run.py [seconds] [modes...]"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
from keyhuntm1cpu_amd.power import PowerSampler  # noqa: E402

BIN = os.path.join(REPO, "tools", "microbench", "valu_energy")
MODES = ["sleep", "nop", "add_u32", "mov_b32", "alignbit", "addc_vcc", "mad64", "mad_addc", "fma_f64", "stream",
         "gather_l2", "gather_mall", "gather_hbm", "salu", "smem", "lds", "scratch", "scratch_l2", "sleep"]


def main():
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 4.0
    modes = sys.argv[2:] or MODES
    base = None
    for m in modes:
        with PowerSampler(period=0.05) as ps:
            r = subprocess.run([BIN, m, str(secs)], capture_output=True, text=True, timeout=120)
        if r.returncode:
            print(r.stdout + r.stderr, file=sys.stderr)
            sys.exit(r.returncode)
        line = json.loads(r.stdout.strip().splitlines()[-1])
        sm = ps.summary()
        w = sm.get("power_w_from_energy") or sm.get("power_w_avg")
        line.update({"power_w": w, "gfxclk_mhz": sm.get("gfxclk_mhz_avg"), "ppt": sm.get("ppt_residency_frac")})
        if m == "sleep" and base is None:
            base = w
        if base is not None and w is not None and m != "sleep":
            line["pj_per_unit_above_sleep"] = round((w - base) / line["units_per_s"] * 1e12, 3)
            line["pj_per_unit_total"] = round(w / line["units_per_s"] * 1e12, 3)
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
