"""Diagnostic: wave timeline of the frontier kernel (stamped library): per wave
(episode) its start / end (s_memrealtime, 100 MHz), SIMD / CU / XCD, slots.
Config-3 shape: 5 x P individuals x (4560-tick training + 912-tick validation
episode), H=32, episodes in the GA session's order."""
import ctypes
import os
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
os.environ["SGMM_LIB"] = str(ROOT / "tools/stamps/libsgmm_stamps.so")
os.environ["SGMM_TABLE_PATH"] = "frontier"
sys.path.insert(0, str(ROOT))
import numpy as np
import torch
import sgmm_pkg
sg = sgmm_pkg.load()
from sgmm_amd import _lib, synthetic
L = _lib.load()
L.sgmm_debug_frontier_tstamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
L.sgmm_debug_frontier_thwid.argtypes = [ctypes.c_void_p, ctypes.c_int]
H, K = 32, 5
P = int(sys.argv[1]) if len(sys.argv) > 1 else 512
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
eb = sg.EpisodeBatch(np.array(gen), offs, lens, np.zeros(n)).to(dev)
eng = sg.RolloutEngine(dev)
for _ in range(3):
    eng.fitness(ticks, eb, params, pop, H)
torch.cuda.synchronize()
h = np.zeros((n, 8), np.uint64)
L.sgmm_debug_frontier_tstamps(h.ctypes.data, n)
hw = np.zeros((n, 2), np.uint32)
L.sgmm_debug_frontier_thwid(hw.ctypes.data, n)
t0 = h[:, 0].astype(np.int64); t1 = h[:, 1].astype(np.int64)
base = t0.min()
s, e_ = (t0 - base) * 10, (t1 - base) * 10  # ns
dur = e_ - s
simd = (hw[:, 0] >> 4) & 3; cu = (hw[:, 0] >> 8) & 15; se = (hw[:, 0] >> 13) & 7; xcc = hw[:, 1] & 7
sid = ((xcc * 8 + se) * 16 + cu) * 4 + simd
lens = np.array(lens)
print(f"waves {n}; kernel span {e_.max() / 1e3:.1f} us; distinct SIMDs {len(np.unique(sid))}")
for name, m in (("train", lens == 4560), ("val", lens == 912)):
    if not m.any():
        continue
    print(f"  {name}: duration med {np.median(dur[m]) / 1e3:.1f} us p10 {np.percentile(dur[m], 10) / 1e3:.1f} "
          f"p90 {np.percentile(dur[m], 90) / 1e3:.1f}; start med {np.median(s[m]) / 1e3:.1f} us "
          f"max {s[m].max() / 1e3:.1f}; slots/wave {np.median(h[m, 2]):.0f} tile-slots {np.median(h[m, 3]):.0f}")
# per-SIMD busy: sum of wave durations and concurrency
u, inv = np.unique(sid, return_inverse=True)
busy = np.bincount(inv, weights=dur)
cnt = np.bincount(inv)
last = np.zeros(len(u)); np.maximum.at(last, inv, e_)
print(f"  waves per SIMD: mean {cnt.mean():.2f} max {cnt.max()}; per-SIMD sum of wave time / span: "
      f"med {np.median(busy / last):.2f}; SIMD last end: med {np.median(last) / 1e3:.1f} us max {last.max() / 1e3:.1f}")
# concurrency histogram over time
grid = np.linspace(0, e_.max(), 40)
act = [(np.sum((s <= t) & (e_ > t))) for t in grid]
print("  resident waves over time (/1024 SIMDs):", [round(a / 1024, 2) for a in act[::4]])
# per-SIMD wave count vs when the SIMD finishes
for c in np.unique(cnt):
    m = cnt == c
    print(f"  SIMDs with {c} waves: {m.sum():4d}; last end med {np.median(last[m]) / 1e3:.1f} us "
          f"max {last[m].max() / 1e3:.1f}; wave duration med {np.median(dur[np.isin(inv, np.where(m)[0])]) / 1e3:.1f} us")
cu_id = sid // 4
uc, cinv = np.unique(cu_id, return_inverse=True)
ccnt = np.bincount(cinv)
print("  waves per CU: " + " ".join(f"{c}:{(ccnt == c).sum()}" for c in np.unique(ccnt)))
xc = np.bincount(xcc, minlength=8)
print("  waves per XCD:", list(xc))
r = np.corrcoef(h[:, 2].astype(float), dur)[0, 1]
print(f"  corr(slots, duration) {r:.2f}")
sl = h[:, 2].astype(float)
print("  slots/wave percentiles 50/90/99/max:", [float(np.percentile(sl, p)) for p in (50, 90, 99)], float(sl.max()))
top = np.argsort(-e_)[:12]
print("  last-ending waves: (end us, dur us, slots, waves on its SIMD)")
for w in top:
    print(f"    {e_[w] / 1e3:7.1f} {dur[w] / 1e3:7.1f} {int(sl[w]):5d} {cnt[inv[w]]}")
hs = np.argsort(-sl)[:8]
print("  heaviest waves: (slots, dur us, end us, waves on SIMD)", [(int(sl[w]), round(dur[w] / 1e3, 1), round(e_[w] / 1e3, 1), int(cnt[inv[w]])) for w in hs])
# is a SIMD's end set by the matrix work on it?  per-SIMD slot total vs its last end
simd_slots = np.bincount(inv, weights=sl)
A = np.vstack([simd_slots, np.ones_like(simd_slots)]).T
coef, *_ = np.linalg.lstsq(A, last / 1e3, rcond=None)
print(f"  per-SIMD slots: mean {simd_slots.mean():.0f} max {simd_slots.max():.0f}; last end ~ {coef[0]:.3f} us/slot "
      f"+ {coef[1]:.1f} us, corr {np.corrcoef(simd_slots, last)[0, 1]:.2f}")
for lo, hi in ((0, 200), (200, 260), (260, 320), (320, 400), (400, 2000)):
    m = (simd_slots >= lo) & (simd_slots < hi)
    if m.any():
        print(f"    SIMDs with {lo}-{hi} slots: {m.sum():4d}, last end med {np.median(last[m]) / 1e3:.1f} max {last[m].max() / 1e3:.1f} us")
# what packing the (chunk, state) pairs densely into the 64 columns would save
pk = h[:, 4].astype(float); pt = h[:, 5].astype(float); ts = h[:, 3].astype(float)
for name, m in (("train", lens == 4560), ("val", lens == 912)):
    if not m.any():
        continue
    print(f"  packed {name}: slots {sl[m].sum():.0f} -> {pk[m].sum():.0f}, tile-slots {ts[m].sum():.0f} -> {pt[m].sum():.0f}")
hs = np.argsort(-sl)[:16]
print("  heaviest waves (slots, packed slots, tile-slots, packed tile-slots):",
      [(int(sl[w]), int(pk[w]), int(ts[w]), int(pt[w])) for w in hs])
for q in (50, 90, 99):
    w = np.argsort(sl)[int(len(sl) * q / 100) - 1]
    print(f"  p{q} wave: slots {int(sl[w])} packed {int(pk[w])} tile-slots {int(ts[w])} packed {int(pt[w])}")
