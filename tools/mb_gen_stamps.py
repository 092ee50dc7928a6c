"""Diagnostic: table/scan phase stamps inside the bench generation (asked
population + fused GA step), stamped library build (tools/build_stamps.sh)."""
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
L.sgmm_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
P, H, T, Tv = 64, 16, 3600, 720
tr = synthetic.bundle_510300(T, seed=0)
va = synthetic.bundle_510300(Tv, seed=1, start_ticks=3500)  # bench.py's workload
SEED = int(sys.argv[1]) if len(sys.argv) > 1 else 99
GENS = int(sys.argv[2]) if len(sys.argv) > 2 else 8
st = synthetic.train_stats(tr)
torch.manual_seed(0)
eng = sg.DRLEngine(pop_size=P, phi=1e-4, tick_size=0.001, save_dir="/tmp/mbgen", hidden_dim=H, seed=SEED,
                   verbose=False, use_graph=False)
sess = eng.session(tr, va, st, generations=GENS)
for g in range(GENS):
    sess.step(g)
torch.cuda.synchronize()
nch = (T + 63) // 64
gx = (nch + 3) // 4
n_ep = 2 * P
h = np.zeros((n_ep * gx * 4, 8), np.uint64)
L.sgmm_debug_tstamps(h.ctypes.data, len(h))
slots = []
for e in range(n_ep):
    Te = T if e < P else Tv
    for c in range((Te + 63) // 64):
        slots.append(e * gx * 4 + c)
h = h[slots].astype(np.int64)
d = np.diff(h[:, 0:6], axis=1)
q = lambda a: f"med {np.median(a):.0f} p90 {np.percentile(a, 90):.0f} max {a.max():.0f}"
print(f"table waves={len(slots)}")
print(f"  weights     {q(d[:, 0])}\n  mlp         {q(d[:, 1])}\n  env         {q(d[:, 2])}\n"
      f"  prefix      {q(d[:, 3])}\n  write-drain {q(d[:, 4])}\n  total       {q(h[:, 5] - h[:, 0])}")
real0 = h[:, 7].min()
print(f"  wave start ns: {q((h[:, 7] - real0) * 10)}; last end ns {((h[:, 6] - real0) * 10).max():.0f}")
s = np.zeros((n_ep, 16), np.uint64)
L.sgmm_debug_stamps(s.ctypes.data, n_ep)
s = s.astype(np.int64)
rel = lambda k, sl: np.median(s[sl, k] - s[sl, 0])
print(f"scan (train episodes, median): chunk-starts {rel(1, slice(0, P)):.0f} rewards {rel(2, slice(0, P)):.0f} "
      f"records {rel(9, slice(0, P)):.0f} walk-done {rel(10, slice(0, P)):.0f} end {rel(3, slice(0, P)):.0f}")
print(f"scan walk: iterations med {np.median(s[:P,13]):.0f} max {s[:P,13].max()}, slow med {np.median(s[:P,14]):.0f} max {s[:P,14].max()}")
print(f"scan walk val eps: iterations med {np.median(s[P:,13]):.0f} max {s[P:,13].max()}, slow med {np.median(s[P:,14]):.0f} max {s[P:,14].max()}")
last = np.nonzero(s[:, 5] > s[:, 0])[0]
if len(last):
    k = last[0]
    print(f"generation tail (last-arriving episode {k}): arrival {s[k, 4] - s[k, 0]} cycles after its entry, "
          f"tail {s[k, 5] - s[k, 4]} cycles; first scan entry -> tail end {s[k, 5] - s[:, 0].min()} cycles")
L.sgmm_debug_tail.argtypes = [ctypes.c_void_p]
tl = np.zeros(8, np.uint64)
L.sgmm_debug_tail(tl.ctypes.data)
tl = tl.astype(np.int64)
s4k = np.zeros((4096, 16), np.uint64)
L.sgmm_debug_stamps(s4k.ctypes.data, 4096)
t0 = int(s4k[4095, 0])
print("tail phases (cycles from the ticket): loads", tl[0] - t0, "shuffles", tl[6] - t0, "barrier", tl[7] - t0,
      "argmax", tl[1] - t0, "regen", tl[2] - t0, "barrier", tl[3] - t0, "bookkeeping", tl[4] - t0, "best copy", tl[5] - t0)
dd = s[:, 3] - s[:, 0]
print("scan total cycles per episode: train med", np.median(dd[:P]), "max", dd[:P].max(), "val med", np.median(dd[P:]), "max", dd[P:].max())
hist = sess.hist[:GENS].cpu().numpy().view(sg.drl_engine.HIST_DTYPE).reshape(-1)
print("train_f", hist["train_f"], "val_f", hist["val_f"])
