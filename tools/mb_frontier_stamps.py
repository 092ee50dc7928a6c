"""Diagnostic: per-wave phase cycles of the frontier kernel (stamped library,
tools/build_stamps.sh), on a config-3-shaped batch: P individuals x (one
4560-tick training episode + one 912-tick validation episode), H=32.
Per wave: cycles in layers 1-2 (MFMA issue), relu + transpose (MFMA drain),
layer 3, the FPT step, the per-tick head and the plane writes."""
import ctypes
import os
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
os.environ["SGMM_LIB"] = str(ROOT / os.environ.get("STAMP_LIB", "tools/stamps/libsgmm_phase.so"))
os.environ["SGMM_TABLE_PATH"] = "frontier"
sys.path.insert(0, str(ROOT))
import numpy as np
import torch
import sgmm_pkg
sg = sgmm_pkg.load()
from sgmm_amd import _lib, synthetic
L = _lib.load()
L.sgmm_debug_frontier_tstamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
H = int(os.environ.get("H", 32))
P = int(sys.argv[1]) if len(sys.argv) > 1 else 512
sigma = float(sys.argv[2]) if len(sys.argv) > 2 else 0.05
dev = torch.device("cuda")
tr = synthetic.bundle_510300(4560, seed=0)
va = synthetic.bundle_510300(912, seed=1)
st = synthetic.train_stats(tr)
ticks = sg.TickStore(); s0 = ticks.add(tr, st); s1 = ticks.add(va, st); ticks.to(dev)
params = sg.params_tensor([sg.EnvConfig(phi=1e-3, tick_size=0.001)], dev)
pop = synthetic.population(P, H, sigma=sigma, seed=1).to(dev)
NV = 0 if os.environ.get("TRAIN_ONLY") else P  # TRAIN_ONLY=1: the best-validation training launch
offs = [ticks.segments[s0][0]] * P + [ticks.segments[s1][0]] * NV
lens = [4560] * P + [912] * NV
eb = sg.EpisodeBatch(np.r_[np.arange(P), np.arange(NV)], offs, lens, np.zeros(P + NV)).to(dev)
eng = sg.RolloutEngine(dev)
for _ in range(3):
    eng.fitness(ticks, eb, params, pop, H)
torch.cuda.synchronize()
n = P + NV
h = np.zeros((n, 8), np.uint64)
L.sgmm_debug_frontier_tstamps(h.ctypes.data, n)
h = h.astype(np.float64)
for name, sl, T in (("train", slice(0, P), 4560), ("val", slice(P, P + NV), 912))[:2 if NV else 1]:
    x = h[sl]
    CL = max(4, ((T + 63) // 64 + 3) // 4 * 4)
    med = lambda a: float(np.median(a))
    print(f"{name}: T={T} chunk={CL} waves={len(x)}")
    print(f"  cycles/wave {med(x[:, 0]):9.0f}   per tick {med(x[:, 0]) / CL:7.0f}   wall {med(x[:, 7]) / 100:8.1f} us"
          f"   shader clock {med(x[:, 0] / np.maximum(x[:, 7], 1)) / 10:6.3f} GHz")
    labs = ((1, "L1+L2 issue"), (2, "L2 drain+tr+L3"), (4, "FPT+stores"), (5, "tick head"), (6, "tick tail"))
    if True:
        print(f"  slots/wave {med(x[:, 3]):6.0f}  cycles per slot {med(x[:, 0] / np.maximum(x[:, 3], 1)):7.0f}"
              f"  (L1+L2 issue per slot {med(x[:, 1] / np.maximum(x[:, 3], 1)):6.0f}, drain+L3 per slot "
              f"{med(x[:, 2] / np.maximum(x[:, 3], 1)):6.0f}, FPT per slot {med(x[:, 4] / np.maximum(x[:, 3], 1)):6.0f})")
    for k, lab in labs:
        print(f"  {lab:10s} {med(x[:, k]):9.0f} cyc/wave = {med(x[:, k]) / med(x[:, 0]) * 100:5.1f} %"
              f"   per tick {med(x[:, k]) / CL:6.0f}")
