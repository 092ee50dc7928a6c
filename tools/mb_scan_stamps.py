"""Diagnostic: phase timestamps of the path-scan kernel (stamped library build,
tools/build_stamps.sh).  Slots: 0 entry, 1 chunk starts + trades done, 2 rewards
in LDS, 8 approximate starts, 9 run records, 10 walk done, 3 end; 13/14 walk
iterations / fallback blocks (last window)."""
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
T, H = 3600, 16
dev = torch.device("cuda")
b = synthetic.bundle_510300(T, seed=0)
st = synthetic.train_stats(b)
ticks = sg.TickStore(); ticks.add(b, st); ticks.to(dev)
params = sg.params_tensor([sg.EnvConfig(phi=1e-4, tick_size=0.001)], dev)
eng = sg.RolloutEngine(dev)
for P in (1, 64, 128):
    pop = synthetic.population(P, H, sigma=0.05, seed=1).to(dev)
    eps = sg.EpisodeBatch(np.arange(P), np.zeros(P), np.full(P, T), np.zeros(P)).to(dev)
    for _ in range(3):
        eng.fitness(ticks, eps, params, pop, H)
    torch.cuda.synchronize()
    h = np.zeros((P, 16), np.uint64)
    L.sgmm_debug_stamps(h.ctypes.data, P)
    h = h.astype(np.int64)
    rel = lambda k: np.median(h[:, k] - h[:, 0])
    print(f"P={P}: cycles from entry (median): chunk-starts {rel(1):.0f}, rewards {rel(2):.0f}, "
          f"approx {rel(8):.0f}, records {rel(9):.0f}, walk-done {rel(10):.0f}, end {rel(3):.0f}; "
          f"walk iterations med {np.median(h[:, 13]):.0f} max {h[:, 13].max()}, "
          f"fallback blocks med {np.median(h[:, 14]):.0f} max {h[:, 14].max()}")
