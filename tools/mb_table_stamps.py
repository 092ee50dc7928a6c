"""Diagnostic: per-wave phase timestamps of the policy-table kernel
(stamped library build, tools/build_stamps.sh)."""
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
L.sgmm_debug_tstamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
T, H = int(sys.argv[1]) if len(sys.argv) > 1 else 3600, 16
dev = torch.device("cuda")
b = synthetic.bundle_510300(T, seed=0)
st = synthetic.train_stats(b)
ticks = sg.TickStore(); ticks.add(b, st); ticks.to(dev)
params = sg.params_tensor([sg.EnvConfig(phi=1e-4, tick_size=0.001)], dev)
eng = sg.RolloutEngine(dev)
nch = (T + 63) // 64
gx = (nch + 3) // 4
for P in (1, 64, 128):
    pop = synthetic.population(P, H, sigma=0.05, seed=1).to(dev)
    eps = sg.EpisodeBatch(np.arange(P), np.zeros(P), np.full(P, T), np.zeros(P)).to(dev)
    for _ in range(3):
        eng.fitness(ticks, eps, params, pop, H)
    torch.cuda.synchronize()
    nw = P * gx * 4
    h = np.zeros((nw, 8), np.uint64)
    L.sgmm_debug_tstamps(h.ctypes.data, nw)
    slot = np.array([e * gx * 4 + c for e in range(P) for c in range(nch)])
    h = h[slot].astype(np.int64)
    d = np.diff(h[:, 0:6], axis=1)
    real = (h[:, 7] - h[:, 7].min()) * 10  # ns (100 MHz)
    ghz = (h[:, 5] - h[:, 0]) / ((h[:, 6] - h[:, 7]) * 10.0)
    print(f"  s_memtime rate vs realtime: {np.median(ghz):.3f} GHz; wave wall (ns): "
          f"med {np.median((h[:, 6] - h[:, 7]) * 10):.0f} max {((h[:, 6] - h[:, 7]) * 10).max():.0f}; "
          f"last wave end {((h[:, 6] - h[:, 7].min()) * 10).max():.0f} ns after first start")
    q = lambda a: f"med {np.median(a):.0f} p90 {np.percentile(a, 90):.0f} max {a.max():.0f}"
    print(f"P={P} waves={len(slot)}")
    print(f"  weights     {q(d[:, 0])}\n  mlp         {q(d[:, 1])}\n  env         {q(d[:, 2])}\n"
          f"  prefix      {q(d[:, 3])}\n  write-drain {q(d[:, 4])}\n  total       {q(h[:, 5] - h[:, 0])}")
    print(f"  wave start (ns after first): {q(real)}; "
          f"hist {np.histogram(real, bins=8)[0].tolist()} edges {np.histogram(real, bins=8)[1].astype(int).tolist()}")
