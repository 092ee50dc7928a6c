"""Diagnostic: timeline of the fused frontier launch (stamped library,
tools/build_stamps.sh): per walk its start / end, per scanner its start, first
claim, end, scans and idle polls.  Config-3 shape (5 lambda populations x 512,
H=32, 4560 training ticks), populations trained G generations first."""
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
from sgmm_amd import _lib
from sgmm_amd._lib import stream_ptr
L = _lib.load()
L.sgmm_debug_tstamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
import bench
H, K, P, T = 32, 5, 512, 4560
G_TRAIN = int(sys.argv[1]) if len(sys.argv) > 1 else 10
spec = dict(bench.CONFIGS[3])
data = bench.bundles(spec)
tr = [data[a][0] for _, _, a in spec["pops"]]
va = [data[a][1] for _, _, a in spec["pops"]]
st = [data[a][2] for _, _, a in spec["pops"]]
dev = torch.device("cuda")
eng = bench.make_engine(sg, spec, P, "/tmp/sgmm_ft", None, True, "auto")
sess = eng.session(tr, va, st, generations=G_TRAIN + 1)
sess.steps(0, G_TRAIN)
torch.cuda.synchronize()
ticks = sg.TickStore(); s0 = ticks.add(tr[0], st[0]); ticks.to(dev)
params = sg.params_tensor([sg.EnvConfig(phi=p, tick_size=t) for p, t, _ in spec["pops"]], dev)
Gn = H * H + 7 * H + 2
pop = torch.empty((K * P, Gn), dtype=torch.float32, device=dev)
for k in range(K):
    _lib.check(L.sgmm_ga_ask(ctypes.c_void_p(sess.masters[k].data_ptr()), Gn, ctypes.c_void_p(sess.states[k].data_ptr()),
                             0, int(sess.engs[k].seed), 0, P, ctypes.c_void_p(pop[k * P].data_ptr()), Gn, stream_ptr()),
               "ask")
n = K * P
eb = sg.EpisodeBatch(np.arange(n), np.full(n, ticks.segments[s0][0]), np.full(n, T), np.repeat(np.arange(K), P)).to(dev)
roll = sg.RolloutEngine(dev)
os.environ["SGMM_TABLE_PATH"] = "frontier"
for _ in range(2):
    roll.fitness(ticks, eb, params, pop, H)
torch.cuda.synchronize()
h = np.zeros((65536, 8), np.uint64)
L.sgmm_debug_tstamps(h.ctypes.data, 65536)
w = h[:n].astype(np.int64)
nscan = int(np.count_nonzero(h[32768:32768 + 4096, 0]))
sc = h[32768:32768 + nscan].astype(np.int64)
base = w[:, 0].min()
ws, we = (w[:, 0] - base) / 100, (w[:, 1] - base) / 100
print(f"walks {n}: start max {ws.max():.1f} us, end p10 {np.percentile(we, 10):.0f} p50 {np.median(we):.0f} "
      f"p90 {np.percentile(we, 90):.0f} max {we.max():.0f} us")
s0_, sf, s1 = (sc[:, 0] - base) / 100, (sc[:, 1] - base) / 100, (sc[:, 2] - base) / 100
print(f"scanners {nscan}: start p50 {np.median(s0_):.0f} max {s0_.max():.0f}; first claim p50 {np.median(sf):.0f}; "
      f"end p50 {np.median(s1):.0f} max {s1.max():.0f} us; scans/scanner p50 {np.median(sc[:, 3]):.0f} "
      f"max {sc[:, 3].max()} sum {sc[:, 3].sum()}; polls p50 {np.median(sc[:, 4]):.0f}; "
      f"busy per scan {np.sum(sc[:, 6]) / max(1, sc[:, 3].sum()) / 100:.1f} us")
print("  scanners per XCD", np.bincount(sc[:, 5].astype(int), minlength=8))
grid = np.linspace(0, max(we.max(), s1.max()), 21)
print("  walks resident:", [int(np.sum((ws <= t) & (we > t))) for t in grid])
print("  scans done by t (approx, busy scanners):", [int(np.sum((sf <= t) & (s1 > t))) for t in grid])
np.savez(ROOT / "gpurun_out/fused_timeline.npz", walks=h[:n], scanners=h[32768:32768 + nscan])
