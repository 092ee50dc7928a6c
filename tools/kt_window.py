"""rocprofv3 kernel-trace averages over bench.py's TIMED window.

`rocprofv3 --kernel-trace --stats` averages every dispatch of the process: the
timed run's W warmup + K timed generations, then the eager per-kernel re-run
(W more untimed generations + the profiled ones).  The policy kernel gets cheaper
as the populations train, so that average mixes in the slow early generations.
This takes each kernel's dispatches in start order and averages dispatches
[W, W + K) of its per-generation sequence -- the timed generations -- so the
number is the rocprof measurement of exactly the window the bench line's live
HIP-event mean covers.

    python tools/kt_window.py <kernel_trace.csv> <warmup W> <steps K> [per-gen launches of the kernel=1]
"""
import csv
import sys
from collections import defaultdict


def main():
    path, w, k = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    per = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    rows = defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Kind"] != "KERNEL_DISPATCH":
                continue
            rows[r["Kernel_Name"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Grid_Size_X"])))
    for name, d in sorted(rows.items(), key=lambda kv: -sum(e - s for s, e, _ in kv[1])):
        d.sort()
        # the training launch of a kernel family: its largest grid (validation launches are smaller)
        gmax = max(g for _, _, g in d)
        big = [(s, e) for s, e, g in d if g == gmax]
        if len(big) < (w + k) * per:
            continue
        win = big[w * per:(w + k) * per]
        us = [(e - s) / 1e3 for s, e in win]
        print(f"{name[:90]:90s} grid {gmax:7d}: window mean {sum(us) / len(us):9.1f} us over {len(us)} dispatches "
              f"(first {us[0]:.1f}, last {us[-1]:.1f}); all {len(big)} dispatches {sum((e - s) / 1e3 for s, e in big) / len(big):.1f} us")


if __name__ == "__main__":
    main()
