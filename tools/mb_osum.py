"""Diagnostic: time sgmm_ordered_sum (the episode-sum routine alone) on
reward-like data with HIP events."""
import os
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import numpy as np
import torch
import sgmm_pkg
sg = sgmm_pkg.load()
from sgmm_amd import _lib
L = _lib.load()
rng = np.random.default_rng(11)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 3600
x = np.where(rng.random(n) < 0.4, 0.0, np.where(rng.random(n) < 0.5, -1e-4 * rng.integers(0, 3, n),
                                                rng.normal(1e-3, 1e-3, n)))
xd = torch.from_numpy(x).cuda()
out = torch.zeros(1, dtype=torch.float64, device="cuda")
for _ in range(5):
    L.sgmm_ordered_sum(_lib.ptr(xd), n, 0.0, _lib.ptr(out), _lib.stream_ptr())
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(50):
    L.sgmm_ordered_sum(_lib.ptr(xd), n, 0.0, _lib.ptr(out), _lib.stream_ptr())
e1.record()
torch.cuda.synchronize()
print(os.environ.get("SGMM_LIB", "normal"), "us per call", e0.elapsed_time(e1) * 1e3 / 50,
      "sum", out.item(), "seq", float(np.cumsum(x)[-1]))
