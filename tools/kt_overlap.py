"""Overlap of kernels in a rocprofv3 kernel-trace CSV (multi-stream runs):
prints the dispatches of a window with their queue / stream, start and end
relative to the window, and the fraction of the busy time that had two or
more kernels in flight.

    python tools/kt_overlap.py <kernel_trace.csv> [first_dispatch] [count]
"""
import csv
import sys


def main():
    path = sys.argv[1]
    first = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    count = int(sys.argv[3]) if len(sys.argv) > 3 else 60
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[first:first + count]
    if not rows:
        return
    t0 = int(rows[0]["Start_Timestamp"])
    ev = []
    for r in rows:
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        q = r.get("Queue_Id", r.get("Stream_Id", "?"))
        sid = r.get("Stream_Id", "?")
        name = r["Kernel_Name"].split("(")[0][-48:]
        print(f"{s / 1e3:10.1f} {e / 1e3:10.1f} {(e - s) / 1e3:8.1f} us  q{q} s{sid}  {name}")
        ev += [(s, 1), (e, -1)]
    ev.sort()
    depth, last, busy, multi = 0, 0, 0, 0
    for t, d in ev:
        if depth >= 1:
            busy += t - last
        if depth >= 2:
            multi += t - last
        depth += d
        last = t
    print(f"busy {busy / 1e3:.1f} us, >=2 in flight {multi / 1e3:.1f} us ({100 * multi / max(busy, 1):.0f} %)")


if __name__ == "__main__":
    main()
