"""Diagnostic: adversary path-scan phase cycles (stamped library,
tools/build_stamps.sh) on a config-4-shaped batch: P MM individuals paired
with P adversaries, 3600 ticks, H=32.  Slots (k_path_scan_arl SGMM_STAMP):
0 entry, 1 fill codes in LDS, 6 chunk transducers, 7 chunk starts (pointer
jumping), 11 tick states, 12 rewards gathered, 8/9/10 exact-sum phases of the
last window, 3 record stored.  Usage: python tools/mb_arl_scan_stamps.py [P]"""
import ctypes
import os
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
os.environ["SGMM_LIB"] = str(ROOT / "tools/stamps/libsgmm_stamps.so")
sys.path.insert(0, str(ROOT))
import numpy as np
import torch
import sgmm_pkg
sg = sgmm_pkg.load()
from sgmm_amd import _lib, synthetic
L = _lib.load()
L.sgmm_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
P = int(sys.argv[1]) if len(sys.argv) > 1 else 256
H, T = 32, 3600
dev = torch.device("cuda")
b = synthetic.bundle_510300(T, seed=0)
st = synthetic.train_stats(b)
ticks = sg.TickStore(); seg = ticks.add(b, st); ticks.to(dev)
params = sg.params_tensor([sg.EnvConfig(phi=1e-4, tick_size=0.001)], dev)
pop = synthetic.population(P, H, sigma=0.05, seed=1).to(dev)
adv = synthetic.population(P, 32, sigma=0.05, seed=2).to(dev)
eb = sg.EpisodeBatch(np.arange(P), np.full(P, ticks.segments[seg][0]), np.full(P, T), np.zeros(P)).to(dev)
eng = sg.RolloutEngine(dev)
for _ in range(3):
    eng.fitness(ticks, eb, params, pop, H, adv)
torch.cuda.synchronize()
h = np.zeros((P, 16), np.uint64)
L.sgmm_debug_stamps(h.ctypes.data, P)
h = h.astype(np.int64)
names = [(1, "fills"), (6, "transducers"), (7, "chunk starts"), (11, "tick states"), (12, "gather"),
         (8, "sum a"), (9, "sum b"), (10, "walk"), (3, "end")]
prev = 0
row = []
for k, nm in names:
    v = np.median(h[:, k] - h[:, 0])
    row.append(f"{nm} {v:.0f} (+{v - prev:.0f})")
    prev = v
print(f"adversary scan, {P} episodes x {T} ticks, cycles from entry (median):\n  " + "\n  ".join(row))
tot = (h[:, 3] - h[:, 0]).astype(float)
print(f"  entry->end: p10 {np.percentile(tot, 10):.0f} med {np.median(tot):.0f} max {tot.max():.0f}; "
      f"walk iterations med {np.median(h[:, 13]):.0f}, fallback blocks med {np.median(h[:, 14]):.0f}")
