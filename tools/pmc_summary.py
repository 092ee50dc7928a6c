"""Per-kernel averages of every counter in a directory of rocprofv3 PMC CSVs,
plus the ratios used in DESIGN.md (stall shares, MFMA busy, occupancy).

    python tools/pmc_summary.py <dir> > counters.json

Units (MI355X_MICROARCH.md, constants table): SQ_WAVE_CYCLES / SQ_WAIT_* /
SQ_ACTIVE_INST_* / SQ_BUSY_CYCLES count quad-cycles; SQ_VALU_MFMA_BUSY_CYCLES
counts cycles; GRBM_GUI_ACTIVE is summed over the 8 XCDs.
"""
import collections
import csv
import glob
import json
import re
import sys

KINDS = ("policy_table", "policy_frontier", "path_scan", "ga_step", "rollout_direct", "ordered_sum")


def kind(name):
    for k in KINDS:
        if k in name:
            m = re.search(k + r"(\w*<[^>]*>)?", name)
            return k + (m.group(1).replace(" ", "") if m and m.group(1) else "")
    return name.split("(")[0][:60]


def main(d):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            vals[kind(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, cs in vals.items():
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        avg["_launches"] = max(len(v) for v in cs.values())
        wc = avg.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                      "SQ_WAIT_INST_LDS"):
                if c in avg:
                    avg[f"share_{c}"] = avg[c] / wc
        g = avg.get("GRBM_GUI_ACTIVE")
        if g:
            cyc = g / 8.0  # kernel cycles (sum over 8 XCDs)
            avg["kernel_cycles"] = cyc
            if "SQ_VALU_MFMA_BUSY_CYCLES" in avg:
                # per-SIMD MFMA busy fraction: 1024 SIMDs
                avg["mfma_busy_frac"] = avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024.0 * cyc)
        if wc and "SQ_BUSY_CYCLES" in avg and avg["SQ_BUSY_CYCLES"]:
            # mean resident waves per SE-busy quad-cycle (32 SEs)
            avg["mean_waves_per_cu"] = wc / avg["SQ_BUSY_CYCLES"] / 8.0
        out[k] = avg
    json.dump(out, sys.stdout, indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1])
