"""Per-generation kernel timeline from a rocprofv3 --kernel-trace CSV: for the
last N generations of a graph-replayed bench run, each kernel's duration and
the gap before it (dispatch-to-dispatch idle time on the GPU)."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
short = lambda n: n.split("(")[0].replace("void ", "").replace("sgmm::", "")[:40]
seq = [(short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
# keep only the rollout kernels
seq = [s for s in seq if "policy_table" in s[0] or "path_scan" in s[0]]
tail = seq[-int(sys.argv[2]) * 2 if len(sys.argv) > 2 else -40:]
stats = defaultdict(list)
for prev, cur in zip(tail, tail[1:]):
    stats[cur[0] + " gap before"].append((cur[1] - prev[2]) / 1e3)
for k in tail:
    stats[k[0] + " duration"].append((k[2] - k[1]) / 1e3)
gens = [(b[2] - a[1]) / 1e3 for a, b in zip(tail[0::2], tail[1::2])]
for k, v in sorted(stats.items()):
    v.sort()
    print(f"{k:55s} median {v[len(v)//2]:8.2f} us  min {v[0]:8.2f}  max {v[-1]:8.2f}")
period = [(tail[i + 2][1] - tail[i][1]) / 1e3 for i in range(0, len(tail) - 2, 2)]
period.sort()
print(f"generation period (table start to next table start): median {period[len(period)//2]:.2f} us")
