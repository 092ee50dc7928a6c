"""Diagnostic: per-wave phase cycles of the v3 policy-table kernel (stamped
library, tools/build_stamps.sh).  H=32, one full day (4560 ticks), P in
argv (default 1 64 512).  Slots: 0 start, 1 weights + layer 1 of state 0,
2 all states done, 3 map scan, 4 end; 5 / 6 summed MFMA / vector blocks of
the state loop; 7 realtime at entry."""
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
T, H = int(os.environ.get("T", 4560)), int(os.environ.get("H", 32))
dev = torch.device("cuda")
b = synthetic.bundle_510300(T, seed=0)
st = synthetic.train_stats(b)
ticks = sg.TickStore(); ticks.add(b, st); ticks.to(dev)
params = sg.params_tensor([sg.EnvConfig(phi=1e-4, tick_size=0.001)], dev)
eng = sg.RolloutEngine(dev)
nch = (T + 63) // 64
gx = (nch + 3) // 4
for P in [int(a) for a in sys.argv[1:]] or [1, 64, 512]:
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
    q = lambda a: f"med {np.median(a):7.0f} p10 {np.percentile(a, 10):7.0f} p90 {np.percentile(a, 90):7.0f}"
    real = (h[:, 7] - h[:, 7].min()) * 10
    print(f"P={P} H={H} waves={len(slot)} (cycles per wave)")
    print(f"  weights+layer1(0) {q(h[:, 1] - h[:, 0])}")
    print(f"  state loop        {q(h[:, 2] - h[:, 1])}")
    print(f"    mfma blocks     {q(h[:, 5])}")
    print(f"    vector blocks   {q(h[:, 6])}")
    print(f"  map scan          {q(h[:, 3] - h[:, 2])}")
    print(f"  plane writes      {q(h[:, 4] - h[:, 3])}")
    print(f"  total             {q(h[:, 4] - h[:, 0])}")
    print(f"  wave start (ns after first): {q(real)}")
