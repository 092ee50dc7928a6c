"""Summarise rocprofv3 PMC CSVs into per-kernel HBM traffic per launch.

Correction (MI355X_MICROARCH.md, HBM section): on gfx950 FETCH_SIZE reports
half the bytes of a wide coalesced read, so read bytes = 2 * FETCH_SIZE KiB;
WRITE_SIZE is exact for 16-B streaming stores.  Both counters are KiB.

    python tools/pmc_traffic.py <fetch_dir> <write_dir> <out.json>
"""
import collections
import csv
import glob
import json
import re
import sys

KIND = (("policy_table", "policy_table"), ("policy_frontier", "policy_frontier"), ("path_scan", "path_scan"), ("ga_step", "ga_step"),
        ("ga_ask", "ga_ask"), ("ga_tell", "ga_tell"), ("ga_val_update", "ga_val_update"))


def kind(name):
    """'policy_frontier<32, 5>' style key: family plus template arguments, so the
    main and validation launches of one family are kept apart."""
    for key, k in KIND:
        if key in name:
            m = re.search(key + r"(\w*<[^>]*>)?", name)
            return k + (m.group(1).replace(" ", "") if m and m.group(1) else "")
    return None


def load(d, counter):
    out = collections.defaultdict(list)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = kind(r["Kernel_Name"])
            if k and r["Counter_Name"] == counter:
                out[k].append(float(r["Counter_Value"]))
    return out


def main(fd, wd, out):
    fetch = load(fd, "FETCH_SIZE")
    write = load(wd, "WRITE_SIZE")
    res = {"correction": "read bytes = 2 x FETCH_SIZE (gfx950 half-count on wide reads); KiB units",
           "calibration": "the x2 read correction and exact WRITE_SIZE are calibrated for 16-B-per-lane streams; "
                          "the frontier stores and scan loads are 8 B per lane (uncalibrated), so reads may be "
                          "over-stated up to 2x",
           "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        f = sum(fetch[k]) / len(fetch[k]) if fetch.get(k) else 0.0
        w = sum(write[k]) / len(write[k]) if write.get(k) else 0.0
        res["kernels"][k] = {"fetch_kib": f, "write_kib": w,
                             "hbm_bytes_per_launch": (2 * f + w) * 1024.0,
                             "launches_sampled": len(fetch.get(k, []))}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
