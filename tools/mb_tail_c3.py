"""Diagnostic: the generation tail (tell) in the config-3 training scan --
5 populations x 512, one-wave scan workgroups, best validation -- stamped
library: per population the last-arriving workgroup's tail cycles (slots 4..5)
and its arrival relative to the population's first scan entry."""
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
L.sgmm_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
K, P, H = 5, 512, 32
tr = synthetic.bundle_510300(4560, seed=0)
va = synthetic.bundle_510300(912, seed=1)
st = synthetic.train_stats(tr)
engines = []
for k, phi in enumerate([1e-4, 1e-3, 5e-3, 8e-3, 1e-2]):
    torch.manual_seed(k)
    engines.append(sg.DRLEngine(pop_size=P, phi=phi, tick_size=0.001, save_dir="/tmp/mbtail", hidden_dim=H,
                                seed=100 + k, verbose=False, use_graph=False, val_mode="best"))
m = sg.MultiDRLEngine(engines)
sess = m.session(tr, va, st, generations=4)
for g in range(3):
    sess.step(g)
torch.cuda.synchronize()
h = np.zeros((4096, 16), np.uint64)
L.sgmm_debug_stamps(h.ctypes.data, 4096)
h = h.astype(np.int64)
for k in range(K):
    blk = h[k * P:(k + 1) * P]
    m_ = blk[:, 5] > blk[:, 4]
    if m_.any():
        i = np.where(m_)[0][-1]
        print(f"population {k}: last arriver episode {k * P + i}: tail {blk[i, 5] - blk[i, 4]} cycles; "
              f"its scan {blk[i, 3] - blk[i, 0]} cycles")
