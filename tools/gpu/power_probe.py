"""What the GPU box's amdsmi exposes (raw gpu_metrics fields, energy counter, power cap, BDFs), as JSON.

Run before any HIP work: `python tools/gpu/power_probe.py > gpurun_out/power_probe.json`.
"""
import json

import amdsmi


def clean(v):
    if isinstance(v, dict):
        return {k: clean(x) for k, x in v.items()}
    if isinstance(v, (list, tuple)):
        return [clean(x) for x in v]
    if isinstance(v, (int, float, str, bool)) or v is None:
        return v
    return str(v)


amdsmi.amdsmi_init()
out = {"handles": []}
for h in amdsmi.amdsmi_get_processor_handles():
    d = {}
    for name, f in (("bdf", amdsmi.amdsmi_get_gpu_device_bdf), ("metrics", amdsmi.amdsmi_get_gpu_metrics_info),
                    ("energy", amdsmi.amdsmi_get_energy_count), ("power_cap", amdsmi.amdsmi_get_power_cap_info),
                    ("power_info", amdsmi.amdsmi_get_power_info)):
        try:
            d[name] = clean(f(h))
        except Exception as e:  # noqa: BLE001
            d[name] = {"error": repr(e)}
    out["handles"].append(d)
amdsmi.amdsmi_shut_down()
print(json.dumps(out, indent=1))
