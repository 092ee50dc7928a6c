"""Diagnostic: the frontier spill on GA-TRAINED populations (the state bench.py
times), stamped library (tools/build_stamps.sh): for each spill budget, the
frontier walk timeline (kernel span, SIMD last-end percentiles, the last-ending
walks), the walks that spilled, and the HIP-event times of the frontier, spill and
scan kernels on the same launch.
    python tools/mb_spill_timeline.py [G=15] [config=3] [budgets=0,24,28,32]"""
import ctypes
import os
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
os.environ["SGMM_LIB"] = str(ROOT / os.environ.get("STAMP_LIB", "tools/stamps/libsgmm_stamps.so"))
sys.path.insert(0, str(ROOT))
import numpy as np
import torch

import bench
import sgmm_pkg

sg = sgmm_pkg.load()
from sgmm_amd import _lib
from sgmm_amd.model import genome_size

G_TRAIN = int(sys.argv[1]) if len(sys.argv) > 1 else 15
CONFIG = int(sys.argv[2]) if len(sys.argv) > 2 else 3
BUDGETS = [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "0,24,28,32").split(",")]
SHARD = int(os.environ.get("SHARD", "1"))
L = _lib.load()
L.sgmm_debug_frontier_tstamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
L.sgmm_debug_frontier_thwid.argtypes = [ctypes.c_void_p, ctypes.c_int]
DEV = torch.device("cuda")
spec = dict(bench.CONFIGS[CONFIG])
P, H, T = spec["P"], spec["H"], spec["T"]
if SHARD > 1:
    P = (P + SHARD - 1) // SHARD
K = len(spec["pops"])
Gs = genome_size(H)
data = bench.bundles(spec)
tr = [data[a][0] for _, _, a in spec["pops"]]
va = [data[a][1] for _, _, a in spec["pops"]]
st = [data[a][2] for _, _, a in spec["pops"]]
eng = bench.make_engine(sg, spec, P, tempfile.mkdtemp(), None, True, "auto")
sess = eng.session(tr, va, st, generations=G_TRAIN + 1)
sess.steps(0, G_TRAIN)
torch.cuda.synchronize()
s = _lib.stream_ptr()
pop = torch.empty((K * P, Gs), dtype=torch.float32, device=DEV)
for k, e in enumerate(eng.engines):
    _lib.check(L.sgmm_ga_ask(_lib.ptr(sess.masters[k]), Gs, _lib.ptr(sess.states[k]), 0, e.seed, 0, P,
                             _lib.ptr(pop[k * P:]), Gs, s), "sgmm_ga_ask")
ticks = sg.TickStore()
segs = {a: ticks.segments[ticks.add(data[a][0], data[a][2])] for a in sorted({a for _, _, a in spec["pops"]})}
ticks.to(DEV)
n = K * P
offs = np.concatenate([np.full(P, segs[a][0]) for _, _, a in spec["pops"]])
eps = sg.EpisodeBatch(np.arange(n), offs, np.full(n, T), np.repeat(np.arange(K), P))
if "ORDER" in os.environ:  # the order the walk-order feedback left (a session's walk_order)
    eps.order = sess.walk_order.cpu().numpy()
eps = eps.to(DEV)
params = sg.params_tensor([sg.EnvConfig(phi=phi, tick_size=tick) for phi, tick, _ in spec["pops"]], DEV)
roll = sg.RolloutEngine(DEV)
ref = None
print(f"config {CONFIG} (shard 1/{SHARD}): {K} x {P} episodes of {T} ticks, trained {G_TRAIN} generations")
for bud in BUDGETS:
    _lib.plan_set(spill=bud)
    for _ in range(2):
        f, t = roll.fitness(ticks, eps, params, pop, H)
    torch.cuda.synchronize()
    out = (f.cpu().numpy(), t.cpu().numpy())
    if ref is None:
        ref = out
    same = np.array_equal(ref[0], out[0]) and np.array_equal(ref[1], out[1])
    _lib.profile_read()
    _lib.profile_enable(True)
    for _ in range(3):
        roll.fitness(ticks, eps, params, pop, H)
    kt = _lib.profile_read()
    _lib.profile_enable(False)
    roll.fitness(ticks, eps, params, pop, H)  # the stamped launch
    torch.cuda.synchronize()
    h = np.zeros((32768, 8), np.uint64)
    L.sgmm_debug_frontier_tstamps(h.ctypes.data, 32768)
    hw = np.zeros((32768, 2), np.uint32)
    L.sgmm_debug_frontier_thwid(hw.ctypes.data, 32768)
    rows = np.nonzero(h[:, 1])[0]
    h, hw = h[rows], hw[rows]
    t0, t1 = h[:, 0].astype(np.int64), h[:, 1].astype(np.int64)
    base = t0.min()
    s0, e_ = (t0 - base) * 10, (t1 - base) * 10
    dur = e_ - s0
    sid = ((((hw[:, 1] & 7) * 8 + ((hw[:, 0] >> 13) & 7)) * 16 + ((hw[:, 0] >> 8) & 15)) * 4 + ((hw[:, 0] >> 4) & 3))
    u, inv = np.unique(sid, return_inverse=True)
    last = np.zeros(len(u))
    np.maximum.at(last, inv, e_)
    sl = h[:, 2].astype(float)
    grid = np.linspace(0, e_.max(), 11)
    act = [round(float(np.sum((s0 <= x) & (e_ > x))) / 1024, 2) for x in grid]
    top = np.argsort(-e_)[:6]
    # spilled waves: wspill section of the workspace (the launch's waves = grid of the frontier kernel)
    a256 = lambda x: (x + 255) & ~255
    gm = 2 if (CONFIG == 3 and SHARD == 1) else None
    kms = {k: round(v[0] / v[1] * 1e3, 1) for k, v in kt.items()}
    print(f"spill {bud:3d}: results {'identical' if same else 'DIFFER'}; kernels (us) {kms}; walks {len(rows)} span "
          f"{e_.max() / 1e3:.1f} us; SIMD last end med {np.median(last) / 1e3:.1f} p90 {np.percentile(last, 90) / 1e3:.1f} "
          f"p99 {np.percentile(last, 99) / 1e3:.1f}; resident {act}")
    print("    last-ending walks (end us, dur us, slots):",
          [(round(e_[w] / 1e3, 1), round(dur[w] / 1e3, 1), int(sl[w])) for w in top],
          f"slots p50/p99/max {np.percentile(sl, 50):.0f}/{np.percentile(sl, 99):.0f}/{sl.max():.0f}")
