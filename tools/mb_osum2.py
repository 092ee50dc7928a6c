"""Diagnostic: sgmm_ordered_sum on the bench workload's real selected rewards
(oracle trace of one P=64 bench episode, H=16, T=3600).  Prints us per call
(HIP events) with the stamped library
(SGMM_LIB=tools/stamps/libsgmm_stamps.so) also the v2 phase cycles."""
import ctypes
import os
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "oracle")]
import numpy as np
import torch
import sgmm_pkg
sg = sgmm_pkg.load()
import oracle
from sgmm_amd import _lib, synthetic
L = _lib.load()
T, H = 3600, 16
b = synthetic.bundle_510300(T, seed=0)
st = synthetic.train_stats(b)
pop = synthetic.population(4, H, sigma=0.05, seed=1).numpy()
s1n, s2n = oracle.normalize_signals(b[0], b[1], st)
_, _, tr = oracle.evaluate(pop[0], H, None, s1n, s2n, *b[2:], oracle.params(phi=1e-4, tick=0.001), trace=True)
x = np.ascontiguousarray(tr["reward"], np.float64)
xd = torch.from_numpy(x).cuda()
out = torch.zeros(1, dtype=torch.float64, device="cuda")
call = lambda: L.sgmm_ordered_sum(_lib.ptr(xd), len(x), 0.0, _lib.ptr(out), _lib.stream_ptr())
for _ in range(5):
    call()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(100):
    call()
e1.record()
torch.cuda.synchronize()
seq = 0.0
for v in x:
    seq += v
print(os.path.basename(os.environ.get("SGMM_LIB", "libsgmm.so")),
      "us per call %.2f" % (e0.elapsed_time(e1) * 1e3 / 100), "exact", out.item() == seq)
if "stamps" in os.environ.get("SGMM_LIB", ""):
    L.sgmm_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    h = np.zeros((1, 16), np.uint64)
    L.sgmm_debug_stamps(h.ctypes.data, 1)
    h = h.astype(np.int64)[0]
    print("  cycles: approx->records %d, walk %d; iterations %d fallback %d" % (h[9] - h[8], h[10] - h[9], h[13], h[14]))
