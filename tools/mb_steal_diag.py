"""Diagnostic: the frontier launch with tick hand-offs on / off on config 3's
population after G generations: launch time (HIP events), hand-off counters
(items queued, refused, helpers that left early) and equality of the results."""
import os
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
if os.environ.get("STAMPS"):
    os.environ["SGMM_LIB"] = str(ROOT / "tools/diag/libsgmm_stamps.so")
sys.path.insert(0, str(ROOT))
import ctypes
import numpy as np
import torch
import sgmm_pkg
sg = sgmm_pkg.load()
from sgmm_amd import _lib
from sgmm_amd._lib import stream_ptr
L = _lib.load()
import bench
H, K, P, T = 32, 5, 512, 4560
G_TRAIN = int(sys.argv[1]) if len(sys.argv) > 1 else 5
spec = dict(bench.CONFIGS[3])
data = bench.bundles(spec)
tr = [data[a][0] for _, _, a in spec["pops"]]
va = [data[a][1] for _, _, a in spec["pops"]]
st = [data[a][2] for _, _, a in spec["pops"]]
dev = torch.device("cuda")
eng = bench.make_engine(sg, spec, P, "/tmp/sgmm_sd", None, True, "auto")
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


def a256(x):
    return (x + 255) & ~255


steps = n * T
nchunk = steps // 64 + n + 1
off = a256(max(nchunk, n * 256) * 8) + a256(max(nchunk * 8, n * 256 * 32)) + a256((n * 256 + n) * 4) + \
    a256(4 * 32 * 11 + 4 * 8 * n)
res = {}
MODES = os.environ.get("MODES", "0/4/3/0 1/4/3/0 1/1/3/0").split()
for mode in MODES:  # steal / max segments / checks / helper every (0: default)
    st_, ms_, ck_, ev_ = mode.split("/")
    os.environ["SGMM_FRONTIER_STEAL"] = st_
    os.environ["SGMM_STEAL_MAXSEG"] = ms_
    os.environ["SGMM_STEAL_CHK"] = ck_
    os.environ["SGMM_STEAL_EVERY"] = ev_
    ts = []
    for _ in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        f, t = roll.fitness(ticks, eb, params, pop, H)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ws = roll._ws
    ctl = ws[off:off + 4 * 160].view(torch.int32).cpu().numpy()
    seg = ws[off + 640:off + 640 + 16 * n].view(torch.int32).cpu().numpy().reshape(n, 4)
    print(f"steal={mode}: fitness launch (frontier + scan) {['%.0f' % x for x in ts]} us; queued {ctl[32]} "
          f"head {ctl[0]} active {ctl[64]} idle {ctl[96]} started {ctl[128]} refused {ctl[129]} left-early {ctl[130]} helpers {ctl[131]}; "
          f"segments/episode {np.bincount(np.minimum(seg[:, 0], 4), minlength=5)}", flush=True)
    res.setdefault(mode[0], (f.cpu().numpy(), t.cpu().numpy()))
    if os.environ.get("STAMPS") and st_ == "1":
        L.sgmm_debug_tstamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
        hh = np.zeros((65536, 8), np.uint64); L.sgmm_debug_tstamps(hh.ctypes.data, 65536)
        w = hh[49152:49152 + n].astype(np.int64)
        base = w[:, 0].min()
        st_, we, ex = (w[:, 0] - base) / 100, (w[:, 1] - base) / 100, (w[:, 2] - base) / 100
        print(f"   walk start max {st_.max():.0f}; own walk end p50 {np.median(we):.0f} p90 {np.percentile(we, 90):.0f} "
              f"max {we.max():.0f}; exit p50 {np.median(ex):.0f} max {ex.max():.0f} us; items/wave max {w[:, 3].max()} "
              f"sum {w[:, 3].sum()}; waves with >1 item {np.sum(w[:, 3] > 1)}", flush=True)
        wt = hh[:n].astype(np.int64)  # per-episode walk rows (timeline build: start, end of the last walk of row e)

print("results equal:", np.array_equal(res["0"][0], res["1"][0]) and np.array_equal(res["0"][1], res["1"][1]))
