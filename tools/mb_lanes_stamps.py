"""Diagnostic: phases of the lanes path scan (k_path_scan_lanes) on GA-trained
config-3 populations (stamped library, tools/build_stamps.sh).  Trains config 3
G generations, materializes generation G's population and runs its training
episodes through a fitness launch; per workgroup (8 episodes) prints the cycles of
phase 1 (chunk starts), the first gather, the windows, wave 0's chain and the end.
    python tools/mb_lanes_stamps.py [G=15]"""
import ctypes
import os
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
os.environ["SGMM_LIB"] = str(ROOT / "tools/stamps/libsgmm_stamps.so")
sys.path.insert(0, str(ROOT))
import numpy as np
import torch

import bench
import sgmm_pkg

sg = sgmm_pkg.load()
from sgmm_amd import _lib
from sgmm_amd.model import genome_size

G_TRAIN = int(sys.argv[1]) if len(sys.argv) > 1 else 15
L = _lib.load()
L.sgmm_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
spec = dict(bench.CONFIGS[3])
P, H, T = spec["P"], spec["H"], spec["T"]
K = len(spec["pops"])
G = genome_size(H)
data = bench.bundles(spec)
tr = [data[a][0] for _, _, a in spec["pops"]]
va = [data[a][1] for _, _, a in spec["pops"]]
st = [data[a][2] for _, _, a in spec["pops"]]
eng = bench.make_engine(sg, spec, P, tempfile.mkdtemp(), None, True, "auto")
sess = eng.session(tr, va, st, generations=G_TRAIN + 1)
sess.steps(0, G_TRAIN)
torch.cuda.synchronize()
s = _lib.stream_ptr()
pop = torch.empty((K * P, G), dtype=torch.float32, device="cuda")
for k, e in enumerate(eng.engines):
    _lib.check(L.sgmm_ga_ask(_lib.ptr(sess.masters[k]), G, _lib.ptr(sess.states[k]), 0, e.seed, 0, P,
                             _lib.ptr(pop[k * P:]), G, s), "sgmm_ga_ask")
ticks = sg.TickStore()
seg = {}
for k in range(K):
    if id(tr[k]) not in seg:
        seg[id(tr[k])] = ticks.segments[ticks.add(tr[k], st[k])]
ticks.to("cuda")
offs = np.concatenate([np.full(P, seg[id(tr[k])][0]) for k in range(K)])
eps = sg.EpisodeBatch(np.arange(K * P), offs, np.full(K * P, T), np.repeat(np.arange(K), P)).to("cuda")
params = sg.params_tensor([sg.EnvConfig(phi=phi, tick_size=tick) for phi, tick, _ in spec["pops"]], "cuda")
r = sg.RolloutEngine("cuda")
for _ in range(3):
    r.fitness(ticks, eps, params, pop, H, None)
torch.cuda.synchronize()
nwg = (K * P + 7) // 8
g = np.zeros((4096, 16), np.uint64)
L.sgmm_debug_stamps(g.ctypes.data, 4096)
g = g[:nwg].astype(np.int64)
med = lambda a: float(np.median(a))
p90 = lambda a: float(np.percentile(a, 90))
tot = g[:, 4] - g[:, 0]
for lab, a in (("phase 1 (chunk starts, trades)", g[:, 1] - g[:, 0]), ("first gather", g[:, 2] - g[:, 1]),
               ("windows", g[:, 3] - g[:, 2]), ("  of which wave 0's chains", g[:, 12]), ("records + tail", g[:, 4] - g[:, 3]),
               ("entry -> end", tot)):
    print(f"{lab:32s} med {med(a):9.0f} p90 {p90(a):9.0f} max {a.max():9.0f} cycles")
print(f"span of the launch {g[:, 4].max() - g[:, 0].min()} cycles; workgroup starts: med {med(g[:, 0] - g[:, 0].min()):.0f}"
      f" max {(g[:, 0] - g[:, 0].min()).max()}")
