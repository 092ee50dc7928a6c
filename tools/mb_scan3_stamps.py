"""Diagnostic: path-scan phase cycles on a config-3-shaped batch (stamped
library, frontier chunks): K populations x P individuals x (4560-tick training
+ 912-tick validation episode), H=32.  Slots (sgmm_rollout.hip SGMM_STAMP):
0 entry, 1 chunk starts + trades, 2 rewards of the last window in LDS, 8
approximate starts, 9 run records, 10 walk done, 3 end; 13 / 14 walk
iterations / fallback blocks of the last window."""
import ctypes
import os
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
os.environ["SGMM_LIB"] = str(ROOT / "tools/stamps/libsgmm_stamps.so")
os.environ.setdefault("SGMM_TABLE_PATH", "frontier")
sys.path.insert(0, str(ROOT))
import numpy as np
import torch
import sgmm_pkg
sg = sgmm_pkg.load()
from sgmm_amd import _lib, synthetic
L = _lib.load()
L.sgmm_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
H, K = 32, 5
P = int(sys.argv[1]) if len(sys.argv) > 1 else 400
dev = torch.device("cuda")
tr = synthetic.bundle_510300(4560, seed=0)
va = synthetic.bundle_510300(912, seed=1)
st = synthetic.train_stats(tr)
ticks = sg.TickStore(); s0 = ticks.add(tr, st); s1 = ticks.add(va, st); ticks.to(dev)
params = sg.params_tensor([sg.EnvConfig(phi=1e-3, tick_size=0.001)], dev)
pop = synthetic.population(K * P, H, sigma=0.05, seed=1).to(dev)
gen, offs, lens = [], [], []
VAL = not os.environ.get("TRAIN_ONLY")  # TRAIN_ONLY=1: the best-validation training launch
for k in range(K):
    gen += list(range(k * P, (k + 1) * P)) * (2 if VAL else 1)
    offs += [ticks.segments[s0][0]] * P + ([ticks.segments[s1][0]] * P if VAL else [])
    lens += [4560] * P + ([912] * P if VAL else [])
n = len(gen)
assert n <= 4096
eb = sg.EpisodeBatch(np.array(gen), offs, lens, np.zeros(n)).to(dev)
eng = sg.RolloutEngine(dev)
for _ in range(3):
    eng.fitness(ticks, eb, params, pop, H)
torch.cuda.synchronize()
h = np.zeros((n, 16), np.uint64)
L.sgmm_debug_stamps(h.ctypes.data, n)
h = h.astype(np.int64)
lens = np.array(lens)
for name, m in (("train", lens == 4560), ("val", lens == 912)):
    if not m.any():
        continue
    x = h[m]
    rel = lambda k: np.median(x[:, k] - x[:, 0])
    print(f"{name}: cycles from entry (median): chunk-starts {rel(1):.0f}, last-window rewards {rel(2):.0f}, "
          f"approx {rel(8):.0f}, records {rel(9):.0f}, walk-done {rel(10):.0f}, end {rel(3):.0f}; "
          f"walk iterations med {np.median(x[:, 13]):.0f}, fallback blocks med {np.median(x[:, 14]):.0f}")
    print(f"   entry spread (cycles, memtime): p10 {np.percentile(x[:, 0] - h[:, 0].min(), 10):.0f} "
          f"med {np.median(x[:, 0] - h[:, 0].min()):.0f} max {(x[:, 0] - h[:, 0].min()).max():.0f}")
tot = (h[:, 3] - h[:, 0]).astype(float)
print(f"  entry->end cycles: p10 {np.percentile(tot, 10):.0f} med {np.median(tot):.0f} p90 {np.percentile(tot, 90):.0f} max {tot.max():.0f}")
print(f"  kernel span (memtime cycles): {(h[:, 3].max() - h[:, 0].min()):.0f}")
g = h[:, 11].astype(float); sm = h[:, 12].astype(float); nw_ = h[:, 15].astype(float)
print(f"  per episode summed over {np.median(nw_):.0f} windows: gather med {np.median(g):.0f} cycles, "
      f"exact sum med {np.median(sm):.0f}; chunk starts med {np.median(h[:, 1] - h[:, 0]):.0f}; "
      f"walk iterations med {np.median(h[:, 13]):.0f} fallback blocks med {np.median(h[:, 14]):.0f}")
# the tell in the last-arriving workgroup of each population (generation launches only)
t4, t5 = h[:, 4], h[:, 5]
m = (t5 > t4) & (t4 > 0)
if m.any():
    print("  tail (last arrivers):", [(int(e), int(t5[e] - t4[e])) for e in np.where(m)[0][:8]])
# the slowest episodes: what distinguishes them (walk iterations, fallbacks, gather / sum cycles, windows)
o = np.argsort(tot)[::-1]
print("  slowest episodes: (e, entry->end, gather, sum, walk iters, fallbacks, windows)")
for e in o[:12]:
    print("   ", int(e), int(tot[e]), int(g[e]), int(sm[e]), int(h[e, 13]), int(h[e, 14]), int(h[e, 15]))
for q in (50, 90, 99):
    sel_ = tot >= np.percentile(tot, q)
    print(f"  >= p{q}: mean fallbacks {h[sel_, 14].mean():.1f} iters {h[sel_, 13].mean():.1f} sum {sm[sel_].mean():.0f} gather {g[sel_].mean():.0f}")
print("  corr(entry->end, fallbacks) %.2f, (.., iters) %.2f, (.., gather) %.2f" % (
    np.corrcoef(tot, h[:, 14])[0, 1], np.corrcoef(tot, h[:, 13])[0, 1], np.corrcoef(tot, g)[0, 1]))
