"""Run tools/microbench/f64mul's timing modes (u32 fm_mul vs the v_fma_f64 product) under board-power
sampling: each mode runs as a child process for SECONDS while this process (no HIP: amdsmi only) samples
power, clock and the firmware's power-limit residency.  Prints one JSON line per mode.
Usage: python tools/microbench/f64mul_run.py [seconds]"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
from keyhuntm1cpu_amd.power import PowerSampler  # noqa: E402

BIN = os.path.join(REPO, "tools", "microbench", "f64mul")


def main():
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 5.0
    for kind in ("u32", "f64", "u32", "f64"):
        with PowerSampler(period=0.05) as ps:
            r = subprocess.run([BIN, "time", kind, str(secs)], capture_output=True, text=True, timeout=120)
        if r.returncode:
            print(r.stdout + r.stderr, file=sys.stderr)
            sys.exit(r.returncode)
        line = json.loads(r.stdout.strip().splitlines()[-1])
        sm = ps.summary()
        line["power"] = {k: sm.get(k) for k in ("power_w_avg", "power_w_from_energy", "gfxclk_mhz_avg",
                                               "ppt_residency_frac", "power_cap_w")}
        w = sm.get("power_w_from_energy") or sm.get("power_w_avg")
        if w:
            line["nJ_per_product"] = round(w / (line["G_products_per_s"] * 1e9) * 1e9, 4)
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
