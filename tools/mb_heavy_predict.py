"""Diagnostic: how heavy is each frontier walk, and can it be told early?
Config-3 shape (5 lambda populations x 512, H=32, 4560 training ticks).  The
populations are trained with the normal session for G generations, then the
next generation's asked population is materialised (sgmm_ga_ask) and run
through the stamped frontier kernel: per walk its slots in the first 8 / 16
ticks and in total, start / end time and SIMD.  Writes
gpurun_out/heavy_g{G}.npz for several G."""
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
from sgmm_amd._lib import ptr, stream_ptr
L = _lib.load()
L.sgmm_debug_frontier_tstamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
L.sgmm_debug_frontier_thwid.argtypes = [ctypes.c_void_p, ctypes.c_int]
sys.path.insert(0, str(ROOT))
import bench
H, K, P, T, Tv = 32, 5, 512, 4560, 912
spec = dict(bench.CONFIGS[3])
data = bench.bundles(spec)
tr = [data[a][0] for _, _, a in spec["pops"]]
va = [data[a][1] for _, _, a in spec["pops"]]
st = [data[a][2] for _, _, a in spec["pops"]]
dev = torch.device("cuda")
eng = bench.make_engine(sg, spec, P, "/tmp/sgmm_heavy", None, True, "auto")
gens = [int(g) for g in (sys.argv[1:] or ["0", "5", "15", "30"])]
sess = eng.session(tr, va, st, generations=max(gens) + 1)
ticks = sg.TickStore(); s0 = ticks.add(tr[0], st[0]); ticks.to(dev)
params = sg.params_tensor([sg.EnvConfig(phi=p, tick_size=t) for p, t, _ in spec["pops"]], dev)
G = H * H + 7 * H + 2
eb = sg.EpisodeBatch(np.arange(K * P), np.full(K * P, ticks.segments[s0][0]), np.full(K * P, T),
                     np.repeat(np.arange(K), P)).to(dev)
roll = sg.RolloutEngine(dev)
os.makedirs(ROOT / "gpurun_out", exist_ok=True)
done = 0
for g in gens:
    if g > done:
        sess.steps(done, g - done)
        done = g
    torch.cuda.synchronize()
    pop = torch.empty((K * P, G), dtype=torch.float32, device=dev)
    for k in range(K):
        _lib.check(L.sgmm_ga_ask(ctypes.c_void_p(sess.masters[k].data_ptr()), G,
                                 ctypes.c_void_p(sess.states[k].data_ptr()), 0, int(sess.engs[k].seed), 0, P,
                                 ctypes.c_void_p(pop[k * P].data_ptr()), G, stream_ptr()), "ask")
    os.environ["SGMM_TABLE_PATH"] = "frontier"
    for _ in range(2):
        roll.fitness(ticks, eb, params, pop, H)
    torch.cuda.synchronize()
    del os.environ["SGMM_TABLE_PATH"]
    n = K * P
    L.sgmm_debug_frontier_tstamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    hh = np.zeros((32768, 8), np.uint64); L.sgmm_debug_frontier_tstamps(hh.ctypes.data, 32768)
    hwh = np.zeros((32768, 2), np.uint32); L.sgmm_debug_frontier_thwid(hwh.ctypes.data, 32768)
    split = hh[16384:16384 + n, 0] != 0  # second chunk groups of split episodes (SGMM_FRONTIER_NW=3)
    h = np.concatenate([hh[:n], hh[16384:16384 + n][split]])
    hw = np.concatenate([hwh[:n], hwh[16384:16384 + n][split]])
    hh[:] = 0
    L.sgmm_debug_frontier_tstamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    tag = os.environ.get("TAG", "")
    np.savez(ROOT / f"gpurun_out/heavy{tag}_g{g}.npz", stamps=h, hwid=hw, nsplit=int(split.sum()),
             phis=np.array([p for p, _, _ in spec["pops"]]))
    t0 = h[:, 0].astype(np.int64); t1 = h[:, 1].astype(np.int64)
    span = (t1.max() - t0.min()) * 10 / 1e3
    sl, s8, s16 = h[:, 2].astype(float), h[:, 6].astype(float), h[:, 7].astype(float)
    print(f"gen {g}: span {span:.0f} us; slots p50 {np.median(sl):.0f} p90 {np.percentile(sl, 90):.0f} "
          f"p99 {np.percentile(sl, 99):.0f} max {sl.max():.0f}; corr(s8, total) {np.corrcoef(s8, sl)[0, 1]:.3f} "
          f"corr(s16, total) {np.corrcoef(s16, sl)[0, 1]:.3f}", flush=True)
