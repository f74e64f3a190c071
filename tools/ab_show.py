"""Print value / launch_us / frac of gpurun_out/ab_*.json (newest run first)."""
import glob
import json
import os

for f in sorted(glob.glob("gpurun_out/ab_*.json"), key=os.path.getmtime):
    try:
        d = json.load(open(f))
        print(f"{f[14:-5]:40s} {d['value']:>12,.0f} {d['roofline']['launch_us']:8.1f} us  frac {d['roofline']['frac']:.3f}")
    except Exception as e:  # noqa: BLE001
        print(f, "unreadable", e)
