"""One-line summary of bench.py JSON lines: value, ms per generation, kernel averages, roofline frac, CPU baseline."""
import json
import sys

for f in sys.argv[1:]:
    d = json.load(open(f))
    r = d.get("roofline") or {}
    cpu = d.get("cpu_baseline") or {}
    w = r.get("launch_us_over_timed_window") or {}
    print(f, f"{d['value'] / 1e9:.3f} G", f"{d['ms_per_step'] * 1e3:.1f} us/gen",
          {k: round(v["avg_us"], 1) for k, v in d.get("kernels", {}).items()},
          "frac", round(r.get("frac", 0.0), 4), "first/last", round(w.get("first", 0)), round(w.get("last", 0)),
          "cpu", cpu.get("value"), (cpu.get("pools") or {}).get("pool16", {}).get("seconds"))
