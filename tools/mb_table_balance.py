"""Diagnostic: how the policy-table kernel's waves of the bench workload
(64 train episodes x 3600 ticks + 64 validation episodes x 720 ticks) land on
SIMDs / CUs / XCDs, and the per-SIMD wall time (stamped library build,
tools/build_stamps.sh)."""
import collections
import ctypes
import os
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
os.environ["SGMM_LIB"] = str(ROOT / "tools/diag/libsgmm_stamps.so")
sys.path.insert(0, str(ROOT))
import numpy as np
import torch
import sgmm_pkg
sg = sgmm_pkg.load()
from sgmm_amd import _lib, synthetic
L = _lib.load()
L.sgmm_debug_tstamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
L.sgmm_debug_thwid.argtypes = [ctypes.c_void_p, ctypes.c_int]
T, TV, H, P = 3600, 720, 16, 64
dev = torch.device("cuda")
b = synthetic.bundle_510300(T + TV, seed=0)
st = synthetic.train_stats(b)
ticks = sg.TickStore(); ticks.add(b, st); ticks.to(dev)
params = sg.params_tensor([sg.EnvConfig(phi=1e-4, tick_size=0.001)], dev)
eng = sg.RolloutEngine(dev)
pop = synthetic.population(P, H, sigma=0.05, seed=1).to(dev)
g = np.concatenate([np.arange(P), np.arange(P)])
off = np.concatenate([np.zeros(P), np.full(P, T)])
ln = np.concatenate([np.full(P, T), np.full(P, TV)])
eps = sg.EpisodeBatch(g, off, ln, np.zeros(2 * P)).to(dev)
for _ in range(3):
    eng.fitness(ticks, eps, params, pop, H)
torch.cuda.synchronize()
gx = ((T + 63) // 64 + 3) // 4
nw = 2 * P * gx * 4
h = np.zeros((nw, 8), np.uint64)
hw = np.zeros((nw, 2), np.uint32)
L.sgmm_debug_tstamps(h.ctypes.data, nw)
L.sgmm_debug_thwid(hw.ctypes.data, nw)
slots = [e * gx * 4 + c for e in range(2 * P) for c in range((int(ln[e]) + 63) // 64)]
h = h[slots].astype(np.int64)
hw = hw[slots]
start = (h[:, 7] - h[:, 7].min()) * 10
end = (h[:, 6] - h[:, 7].min()) * 10
hid, xcc = hw[:, 0].astype(np.int64), hw[:, 1].astype(np.int64)
cu = [(int(x), int((v >> 13) & 7), int((v >> 12) & 1), int((v >> 8) & 15)) for v, x in zip(hid, xcc)]
simd = [c + (int((v >> 4) & 3),) for c, v in zip(cu, hid)]
print(f"waves {len(slots)}; last end {end.max():.0f} ns; end med {np.median(end):.0f} p90 {np.percentile(end, 90):.0f}")
for name, keys in (("xcd", [c[0] for c in cu]), ("cu", cu), ("simd", simd)):
    cnt = collections.Counter(keys)
    v = np.array(list(cnt.values()))
    print(f"{name}: {len(cnt)} used; waves per {name}: min {v.min()} med {np.median(v):.0f} max {v.max()}; "
          f"hist {np.bincount(v).tolist()}")
# per-SIMD load vs its last wave end
by = collections.defaultdict(list)
for k, e_ in zip(simd, end):
    by[k].append(e_)
load = collections.defaultdict(list)
for k, v in by.items():
    load[len(v)].append(max(v))
for n in sorted(load):
    print(f"  SIMDs with {n} waves: {len(load[n])}, their last end med {np.median(load[n]):.0f} max {max(load[n]):.0f} ns")
print("start ns hist", np.histogram(start, bins=8)[0].tolist(), np.histogram(start, bins=8)[1].astype(int).tolist())
