"""Board power and clock samples over a timed region (bench.py's `roofline.power`).

A background thread reads the GPU's metrics table through amdsmi (the driver's sysfs/ioctl interface,
not HIP) every `period` seconds: socket power, the graphics clocks, the throttle status and the energy
accumulator.  The average power over the region comes from the energy accumulator's difference when the
board exposes one (exact over the interval), else from the mean of the power samples.  The power cap is
read once.  Nothing here touches the GPU through HIP; if amdsmi is absent or refuses (no permission), the
sampler reports why and the bench line carries `power: {"available": false, ...}`.
"""
from __future__ import annotations

import threading
import time

_NA = (0xFFFF, 0xFFFFFFFF, 0xFFFFFFFFFFFFFFFF, "N/A")


def _num(v):
    if isinstance(v, (list, tuple)):
        vals = [x for x in (_num(y) for y in v) if x is not None]
        return vals or None
    if v in _NA or v is None:
        return None
    try:
        return float(v)
    except (TypeError, ValueError):
        return None


def _bdf_key(bdf: str) -> tuple[int, int, int] | None:
    """(domain, bus, device) of "dddd:bb:dd[.f]" (amdsmi's BDF and bench.physical_gpu's PCI address)."""
    try:
        dom, bus, rest = bdf.strip().split(":")
        return int(dom, 16), int(bus, 16), int(rest.split(".")[0], 16)
    except (AttributeError, ValueError):
        return None


def _handle_for_bdf(amdsmi, bdf: str | None):
    """The amdsmi handle of the GPU at PCI address `bdf` ("dddd:bb:dd", the full domain:bus:device).  No
    match is an error (the power block is then unavailable), never another GPU's handle; with no address given only a
    one-GPU system has an unambiguous handle."""
    hs = amdsmi.amdsmi_get_processor_handles()
    if not hs:
        return None, "no amdsmi GPU handles"
    want = _bdf_key(bdf) if bdf else None
    if want is None:
        if len(hs) == 1:
            return hs[0], None
        return None, "no PCI address for this rank's GPU and %d amdsmi handles" % len(hs)
    for h in hs:
        try:
            if _bdf_key(amdsmi.amdsmi_get_gpu_device_bdf(h)) == want:
                return h, None
        except Exception:                                  # noqa: BLE001 - a handle we cannot read is skipped
            continue
    return None, "no amdsmi handle at PCI %s" % bdf


class PowerSampler:
    """with PowerSampler(bdf) as ps: <timed region>;  ps.summary() -> dict.  bdf: the GPU's "dddd:bb:dd"."""

    def __init__(self, bdf: str | None = None, period: float = 0.05):
        self.period = period
        self.samples = []
        self.err = None
        self.cap_w = None
        self._stop = threading.Event()
        self._th = None
        self._e0 = self._e1 = None
        try:
            import amdsmi
            amdsmi.amdsmi_init()
            self.amdsmi = amdsmi
            self.h, note = _handle_for_bdf(amdsmi, bdf)
            if self.h is None:
                self.err = note
            else:
                self.note = note
                try:
                    cap = amdsmi.amdsmi_get_power_cap_info(self.h)
                    c = _num(cap.get("power_cap"))
                    self.cap_w = c / 1e6 if c and c > 1e4 else c           # reported in uW on ROCm 6+
                    self.cap_info = {k: _num(v) for k, v in cap.items()}
                except Exception as e:                     # noqa: BLE001
                    self.cap_info = {"error": repr(e)}
        except Exception as e:                             # noqa: BLE001 - amdsmi missing / no permission
            self.amdsmi = None
            self.err = repr(e)

    @classmethod
    def disabled(cls, why: str):
        ps = cls.__new__(cls)
        ps.period, ps.samples, ps.err, ps.cap_w, ps.amdsmi = 0.0, [], why, None, None
        ps._stop, ps._th, ps._e0, ps._e1 = threading.Event(), None, None, None
        return ps

    def _metrics(self):
        m = self.amdsmi.amdsmi_get_gpu_metrics_info(self.h)
        return {"t": time.perf_counter(),
                "power_w": _num(m.get("current_socket_power")) or _num(m.get("average_socket_power")),
                "gfxclk": _num(m.get("current_gfxclk")) or _num(m.get("average_gfxclk_frequency")),
                "gfx_activity": _num(m.get("average_gfx_activity")),
                "temp_hotspot": _num(m.get("temperature_hotspot")),
                "temp_mem": _num(m.get("temperature_mem")),
                "throttle": m.get("throttle_status"),
                "indep_throttle": m.get("indep_throttle_status")}

    _RESIDENCY = ("ppt_residency_acc", "socket_thm_residency_acc", "vr_thm_residency_acc", "hbm_thm_residency_acc",
                  "prochot_residency_acc")

    def _residency(self):
        """The firmware's throttle-residency accumulators and their tick counter (gpu_metrics v1.8): the
        share of the interval spent limited by package power (PPT), temperature or PROCHOT."""
        m = self.amdsmi.amdsmi_get_gpu_metrics_info(self.h)
        r = {k: _num(m.get(k)) for k in self._RESIDENCY + ("accumulation_counter",)}
        return r if r["accumulation_counter"] is not None else None

    def _energy(self):
        """(seconds, joules) from the board's energy accumulator and its stated resolution (uJ per count)."""
        e = self.amdsmi.amdsmi_get_energy_count(self.h)
        return time.perf_counter(), e["energy_accumulator"] * e["counter_resolution"] * 1e-6

    def _run(self):
        while not self._stop.is_set():
            try:
                self.samples.append(self._metrics())
            except Exception as e:                         # noqa: BLE001
                self.err = repr(e)
                return
            self._stop.wait(self.period)

    def __enter__(self):
        if self.amdsmi is not None and self.err is None:
            try:
                self._metrics()
            except Exception as e:                         # noqa: BLE001
                self.err = repr(e)
                return self
            try:
                self._e0 = self._energy()
            except Exception as e:                         # noqa: BLE001
                self.energy_err = repr(e)
            try:
                self._r0 = self._residency()
            except Exception:                              # noqa: BLE001
                self._r0 = None
            self._th = threading.Thread(target=self._run, daemon=True)
            self._th.start()
        return self

    def __exit__(self, *exc):
        if self._th is not None:
            self._stop.set()
            self._th.join()
            if self._e0 is not None:
                try:
                    self._e1 = self._energy()
                except Exception as e:                     # noqa: BLE001
                    self.energy_err = repr(e)
            try:
                self._r1 = self._residency() if getattr(self, "_r0", None) else None
            except Exception:                              # noqa: BLE001
                self._r1 = None
        if self.amdsmi is not None:
            try:
                self.amdsmi.amdsmi_shut_down()
            except Exception:                              # noqa: BLE001
                pass
        return False

    def summary(self, work_units: float | None = None, seconds: float | None = None,
                unit: str = "giant steps") -> dict:
        """Average power, clock and throttle state over the region; joules per 1e9 work units if given
        (average power x `seconds`, the timed region's length)."""
        if self.err and not self.samples:
            return {"available": False, "error": self.err}
        s = self.samples
        out = {"available": True, "samples": len(s), "period_s": self.period, "power_cap_w": self.cap_w}
        pw = [x["power_w"] for x in s if isinstance(x["power_w"], float)]
        # per-XCD clocks come as a list: average over XCDs, then over samples
        clk = []
        for x in s:
            c = x["gfxclk"]
            if isinstance(c, list):
                c = sum(c) / len(c)
            if isinstance(c, float):
                clk.append(c)
        if pw:
            out.update({"power_w_avg": round(sum(pw) / len(pw), 1), "power_w_max": round(max(pw), 1),
                        "power_w_min": round(min(pw), 1)})
        if clk:
            out.update({"gfxclk_mhz_avg": round(sum(clk) / len(clk), 1), "gfxclk_mhz_min": round(min(clk), 1),
                        "gfxclk_mhz_max": round(max(clk), 1)})
        act = [x["gfx_activity"] for x in s if isinstance(x["gfx_activity"], float)]
        if act:
            out["gfx_activity_pct_avg"] = round(sum(act) / len(act), 1)
        th = [x["temp_hotspot"] for x in s if isinstance(x["temp_hotspot"], float)]
        if th:
            out["temp_hotspot_c_max"] = th and max(th)
        thr = sorted({str(x["throttle"]) for x in s if x["throttle"] not in (None, "N/A")})
        if thr:
            out["throttle_status_seen"] = thr[:8]
        ithr = sorted({str(x["indep_throttle"]) for x in s if x["indep_throttle"] not in (None, "N/A")})
        if ithr:
            out["indep_throttle_status_seen"] = ithr[:8]
        e0, e1 = self._e0, self._e1
        if e0 and e1 and e1[0] > e0[0]:
            de, dt = e1[1] - e0[1], e1[0] - e0[0]
            if de > 0:
                out["power_w_from_energy"] = round(de / dt, 1)
                out["energy_j"] = round(de, 2)
        elif getattr(self, "energy_err", None):
            out["energy_error"] = self.energy_err
        r0, r1 = getattr(self, "_r0", None), getattr(self, "_r1", None)
        if r0 and r1 and r1["accumulation_counter"] > r0["accumulation_counter"]:
            ticks = r1["accumulation_counter"] - r0["accumulation_counter"]
            for k in self._RESIDENCY:
                if r0.get(k) is not None and r1.get(k) is not None:
                    out[k.replace("_acc", "_frac")] = round((r1[k] - r0[k]) / ticks, 4)
        if self.cap_w and "power_w_avg" in out:
            out["at_cap_frac"] = round(out["power_w_avg"] / self.cap_w, 3)
        if work_units and seconds and "power_w_avg" in out:
            w = out.get("power_w_from_energy") or out["power_w_avg"]
            out["joules_per_1e9_" + unit.replace(" ", "_")] = round(w * seconds / (work_units / 1e9), 3)
        if getattr(self, "note", None):
            out["note"] = self.note
        return out
