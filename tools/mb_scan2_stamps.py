"""Diagnostic: path-scan phase cycles at BASELINE config 2 (64 individuals,
H=16, 3600-tick training + 720-tick validation episodes, fused validation,
table path, the generation tail in the scan).  Stamped library
(tools/build_stamps.sh); eager generations, the stamps of the last one.
Slots (sgmm_rollout.hip SGMM_STAMP): 0 entry, 1 chunk starts + trades, 2
rewards of the last window in LDS, 8 approximate starts, 9 run records, 10
walk done, 3 end; 4 / 5 tail start / end in the last arriver."""
import argparse
import ctypes
import os
import sys
import tempfile
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
os.environ["SGMM_LIB"] = os.environ.get("STAMP_LIB", str(ROOT / "tools/diag/libsgmm_stamps.so"))
sys.path.insert(0, str(ROOT))
import numpy as np
import torch
import bench
import sgmm_pkg
sg = sgmm_pkg.load()
from sgmm_amd import _lib
L = _lib.load()
L.sgmm_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
ap = argparse.ArgumentParser()
ap.add_argument("--gens", type=int, default=4)
ap.add_argument("bench_args", nargs="*")
a = ap.parse_args()
sys.argv = ["bench.py", "--config", "2"] + a.bench_args
args = bench.parse()
spec = bench.workload_spec(args)
data = bench.bundles(spec)
tr = [data[x][0] for _, _, x in spec["pops"]]
va = [data[x][1] for _, _, x in spec["pops"]]
st = [data[x][2] for _, _, x in spec["pops"]]
eng = bench.make_engine(sg, spec, spec["P"], tempfile.mkdtemp(), None, False, args.val_mode)
sess = eng.session(tr, va, st, generations=a.gens)
sess.steps(0, a.gens)
torch.cuda.synchronize()
n = 2 * spec["P"] * len(spec["pops"])
h = np.zeros((4096, 16), np.uint64)
L.sgmm_debug_stamps(h.ctypes.data, 4096)
tail = int(h[4095, 0])
h = h[:n].astype(np.int64)
t0 = h[:, 0].min()
T = spec["T"]
for name, m in (("train", np.arange(n) % (2 * spec["P"]) < spec["P"]), ("val", np.arange(n) % (2 * spec["P"]) >= spec["P"])):
    x = h[m]
    rel = lambda k: np.median(x[:, k] - x[:, 0])
    print(f"{name}: entry med {np.median(x[:, 0] - t0):.0f} max {(x[:, 0] - t0).max():.0f}; from entry (median): "
          f"chunk-starts {rel(1):.0f}, window in LDS {rel(2):.0f}, approx {rel(8):.0f}, records {rel(9):.0f}, "
          f"walk-done {rel(10):.0f}, end {rel(3):.0f}; end (abs) med {np.median(x[:, 3] - t0):.0f} max "
          f"{(x[:, 3] - t0).max():.0f}; walk iterations med {np.median(x[:, 13]):.0f}, fallback med "
          f"{np.median(x[:, 14]):.0f}")
last = np.where((h[:, 5] > h[:, 4]) & (h[:, 4] > 0))[0]
for e in last[:4]:
    print(f"tail in workgroup {e}: start {h[e, 4] - t0} end {h[e, 5] - t0} ({h[e, 5] - h[e, 4]} cycles)")
print(f"kernel span (memtime cycles, entries to last end): {(np.maximum(h[:, 3], h[:, 5]).max() - t0)}")
# the table kernel's waves (slot 0 entry, 4 end, memtime; 7 entry in s_memrealtime)
L.sgmm_debug_tstamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
L.sgmm_debug_thwid.argtypes = [ctypes.c_void_p, ctypes.c_int]
nw = 8192
ts = np.zeros((nw, 8), np.uint64); L.sgmm_debug_tstamps(ts.ctypes.data, nw)
hw = np.zeros((nw, 2), np.uint32); L.sgmm_debug_thwid(hw.ctypes.data, nw)
ts = ts.astype(np.int64)
v = np.where(ts[:, 4] > ts[:, 0])[0]
if len(v):
    d = ts[v, 4] - ts[v, 0]
    r = ts[v, 7] - ts[v, 7].min()
    print(f"table: {len(v)} waves; wave duration (memtime) p10 {np.percentile(d, 10):.0f} med {np.median(d):.0f} "
          f"p90 {np.percentile(d, 90):.0f} max {d.max()}; entry spread (realtime ticks) med {np.median(r):.0f} "
          f"max {r.max()}; phases med {[int(np.median(ts[v, k] - ts[v, k - 1])) for k in range(1, 5)]}")
    print(f"   entry (realtime ticks, 10 ns) percentiles 50/75/90/95/99: {np.percentile(r, [50, 75, 90, 95, 99]).round()}, "
          f"waves entering after 2 us: {(r > 200).sum()}; duration of those med {np.median(d[r > 200]) if (r > 200).any() else 0:.0f}")
    cu = (hw[v, 1].astype(np.int64) << 8) | ((hw[v, 0] >> 8) & 0xFF)
    for lo, hi in ((0, 200), (200, 10**9)):
        m = (r >= lo) & (r < hi)
        uc, cc = np.unique(cu[m], return_counts=True)
        print(f"   waves per CU entering in [{lo}, {hi}) ticks: {dict(zip(*np.unique(cc, return_counts=True)))} over {len(uc)} CUs")
    out = os.environ.get("STAMP_OUT")
    if out:
        np.savez(out, ts=ts, hw=hw, h=h)
    simd = (hw[v, 1].astype(np.int64) << 16) | ((hw[v, 0] >> 8) & 0xFF) << 4 | ((hw[v, 0] >> 4) & 3)
    u, c = np.unique(simd, return_counts=True)
    print(f"   waves per SIMD: {dict(zip(*np.unique(c, return_counts=True)))} over {len(u)} SIMDs")
# the last generation's tail phases (ga_step_fused SGMM_TAIL_STAMP, thread 0 of the last arriver)
L.sgmm_debug_tail.argtypes = [ctypes.c_void_p]
gt = np.zeros(8, np.uint64); L.sgmm_debug_tail(gt.ctypes.data)
gt = gt.astype(np.int64)
t4 = tail
print(f"tail phases from the ticket (cycles): loads {gt[0] - t4}, wave argmax {gt[6] - t4}, barrier {gt[7] - t4}, "
      f"merged {gt[1] - t4}, regen {gt[2] - t4}, bookkeeping {gt[4] - t4}")
