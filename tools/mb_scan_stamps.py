"""Diagnostic: phase timestamps of the path-scan kernel (stamped library build)."""
import ctypes
import os
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
os.environ["SGMM_LIB"] = str(ROOT / "tools/mb/libsgmm_stamps.so")
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
for P in (1, 64):
    pop = synthetic.population(P, H, sigma=0.05, seed=1).to(dev)
    eps = sg.EpisodeBatch(np.arange(P), np.zeros(P), np.full(P, T), np.zeros(P)).to(dev)
    for _ in range(3):
        eng.fitness(ticks, eps, params, pop, H)
    torch.cuda.synchronize()
    h = np.zeros((P, 16), np.uint64)
    L.sgmm_debug_stamps(h.ctypes.data, P)
    d = (h[:, 1:6].astype(np.int64) - h[:, [0]].astype(np.int64))
    print(f"P={P}: cycles from kernel start (median over episodes): chunk-starts {np.median(d[:,0]):.0f}, "
          f"words-in-LDS {np.median(d[:,1]):.0f}, rewards gathered {np.median(d[:,2]):.0f}, "
          f"sum done {np.median(d[:,3]):.0f}, end {np.median(d[:,4]):.0f}")
    ds = (h[:, 8:13].astype(np.int64) - h[:, [0]].astype(np.int64))
    print(f"   sum phases: approx sums {np.median(ds[:,0]):.0f}, approx starts {np.median(ds[:,1]):.0f}, "
          f"int steps {np.median(ds[:,2]):.0f}, z-prefix {np.median(ds[:,3]):.0f}, walk {np.median(ds[:,4]):.0f}; "
          f"walk iterations med {np.median(h[:,13]):.0f} max {h[:,13].max()}, slow blocks med {np.median(h[:,14]):.0f} max {h[:,14].max()}, slow-path cycles med {np.median(h[:,15]):.0f}, fast-part cycles med {np.median(h[:,7]):.0f}")
