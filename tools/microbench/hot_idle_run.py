"""Static power against die temperature (round 6, VERDICT r5 item 5's unexplained energy): board power of the
`sleep` mode of tools/microbench/valu_energy.hip (every wave resident, sleeping) right after the product kernel has
heated the die, against the same mode on a cool die.  One amdsmi sampler (no HIP in this process) runs over:
  cold sleep (S s) -> the driver's bench command as the heater (H steps, no CPU baseline) -> hot sleep (S s),
and the samples are binned per 0.5 s with the hotspot / memory temperatures, so the decay of the idle power with
the die's cooling is read directly.  The difference between hot and cold idle at the product's temperature is the
static (leakage) part of the product's energy per giant step that no instruction-class microbenchmark sees.
Usage: python tools/microbench/hot_idle_run.py [sleep_s] [heater_steps] > out.json"""
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
from keyhuntm1cpu_amd.power import PowerSampler  # noqa: E402

BIN = os.path.join(REPO, "tools", "microbench", "valu_energy")


def bins(samples, t0, t1, width=0.5):
    out = []
    t = t0
    while t < t1:
        xs = [x for x in samples if t <= x["t"] < t + width]
        pw = [x["power_w"] for x in xs if isinstance(x["power_w"], float)]
        th = [x["temp_hotspot"] for x in xs if isinstance(x["temp_hotspot"], float)]
        tm = [x["temp_mem"] for x in xs if isinstance(x["temp_mem"], float)]
        if pw:
            out.append({"t": round(t - t0, 2), "power_w": round(sum(pw) / len(pw), 1),
                        "hotspot_c": round(sum(th) / len(th), 1) if th else None,
                        "mem_c": round(sum(tm) / len(tm), 1) if tm else None})
        t += width
    return out


def main():
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 8.0
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    marks = {}
    with PowerSampler(period=0.05) as ps:
        marks["cold0"] = time.perf_counter()
        subprocess.run([BIN, "sleep", str(secs)], check=True, capture_output=True, timeout=120)
        marks["cold1"] = marks["heat0"] = time.perf_counter()
        r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", str(steps), "--warmup", "2",
                            "--no-cpu-baseline", "--no-power"], capture_output=True, text=True, timeout=600)
        if r.returncode:
            print(r.stderr[-2000:], file=sys.stderr)
            sys.exit(r.returncode)
        marks["heat1"] = marks["hot0"] = time.perf_counter()
        subprocess.run([BIN, "sleep", str(secs)], check=True, capture_output=True, timeout=120)
        marks["hot1"] = time.perf_counter()
    s = ps.samples
    bench = json.loads(r.stdout.strip().splitlines()[-1])
    heat = bins(s, marks["heat0"], marks["heat1"], 2.0)
    out = {"sleep_s": secs, "heater": "bench.py --steps %d (the product kernel)" % steps, "bench_value": bench["value"],
           "cold_sleep": bins(s, marks["cold0"], marks["cold1"]), "heater_2s_bins": heat,
           "hot_sleep": bins(s, marks["hot0"], marks["hot1"])}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
