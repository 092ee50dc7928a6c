"""Diagnostic: which episodes should the frontier kernel split?  Pass 1 (stamped
library, SGMM_FRONTIER_NW=1) records each training walk's slot count; pass 2
times the normal library (hipEvents) on the config-3 training batch with the
default order (the last 512 of the longest-first order split) and with an
order that puts the heaviest 512 walks in the split positions."""
import ctypes
import os
import subprocess
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import numpy as np

H, K, P = 32, 5, 512
MODE = sys.argv[1] if len(sys.argv) > 1 else "time"
if MODE == "slots":
    os.environ["SGMM_LIB"] = str(ROOT / "tools/stamps/libsgmm_stamps.so")
    os.environ["SGMM_FRONTIER_NW"] = "1"
import torch
import sgmm_pkg
sg = sgmm_pkg.load()
from sgmm_amd import _lib, synthetic
dev = torch.device("cuda")
tr = synthetic.bundle_510300(4560, seed=0)
st = synthetic.train_stats(tr)
ticks = sg.TickStore(); s0 = ticks.add(tr, st); ticks.to(dev)
params = sg.params_tensor([sg.EnvConfig(phi=1e-3, tick_size=0.001)], dev)
pop = synthetic.population(K * P, H, sigma=float(os.environ.get("SIGMA", "0.05")), seed=1).to(dev)
n = K * P
eb = sg.EpisodeBatch(np.arange(n), [ticks.segments[s0][0]] * n, [4560] * n, np.zeros(n)).to(dev)
eng = sg.RolloutEngine(dev)
if MODE == "slots":
    L = _lib.load()
    L.sgmm_debug_frontier_tstamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    eng.fitness(ticks, eb, params, pop, H)
    torch.cuda.synchronize()
    h = np.zeros((n, 8), np.uint64)
    L.sgmm_debug_frontier_tstamps(h.ctypes.data, n)
    np.save("/tmp/frontier_slots.npy", h[:, 2].astype(np.int64))
    print("slots p50/p90/p99/max", np.percentile(h[:, 2], [50, 90, 99]).tolist(), int(h[:, 2].max()))
    sys.exit(0)
slots = np.load("/tmp/frontier_slots.npy")
def timeit(order, reps=6):
    eb.dev["order"] = torch.from_numpy(order.astype(np.int32)).to(dev)
    f0 = eng.fitness(ticks, eb, params, pop, H)
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); eng.fitness(ticks, eb, params, pop, H); b.record(); torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return np.median(ts), f0
base = np.arange(n)
asc = np.argsort(slots, kind="stable")            # lightest first: the heaviest 512 land in the split positions
desc = asc[::-1].copy()                           # heaviest first: the heaviest are whole
t0, f0 = timeit(base)
t1, f1 = timeit(asc)
t2, f2 = timeit(desc)
assert torch.equal(f0[0], f1[0]) and torch.equal(f0[0], f2[0])
print(f"fitness launch (policy + scan): default order {t0:.1f} us, heaviest split {t1:.1f} us, heaviest whole {t2:.1f} us")
# a cheap predictor: each individual's policy at inventory 0 on 64 sampled ticks
# (sgmm_policy_forward), FPT fills from those quotes; score = sampled ticks
# without a fill.  Does ordering by it recover the "heaviest whole" gain?
idx = np.linspace(0, 4559, 64).astype(np.int64)
s1n, s2n = sg.normalize_signals(tr[0], tr[1], st)
states = torch.tensor(np.stack([np.tile(s1n[idx], n), np.tile(s2n[idx], n), np.zeros(64 * n, np.float32)], 1),
                      dtype=torch.float32, device=dev)
gidx = torch.arange(n, dtype=torch.int32, device=dev).repeat_interleave(64)
raw = sg.policy_forward(pop, H, states, gidx).cpu().numpy().reshape(n, 64, 2)
off = np.rint(raw.astype(np.float64) * 5.0)
ask, bid, bmax, smin = (np.asarray(tr[k])[idx] for k in (3, 4, 5, 6))
qa = ask[None, :] + off[:, :, 0] * 0.001
qb = bid[None, :] - off[:, :, 1] * 0.001
fill = (qb >= smin[None, :]) | (qa <= bmax[None, :])
score = (~fill).sum(1)
r = np.corrcoef(score, slots)[0, 1]
pred = np.argsort(-score, kind="stable")
t3, f3 = timeit(pred)
assert torch.equal(f0[0], f3[0])
print(f"predictor corr(no-fill samples, slots) {r:.2f}; ordered by the predictor {t3:.1f} us")
# predictor 2: the share of sampled ticks whose one-step transition map over
# the 5 inventory states is injective (no two paths can merge there)
S = 128
idx = np.linspace(0, 4559, S).astype(np.int64)
invs = np.arange(-2, 3)
x = np.stack([np.tile(np.repeat(s1n[idx], 5), n), np.tile(np.repeat(s2n[idx], 5), n),
              np.tile(np.tile(invs / 2.0, S), n)], 1).astype(np.float32)
states = torch.tensor(x, device=dev)
gidx = torch.arange(n, dtype=torch.int32, device=dev).repeat_interleave(5 * S)
raw = sg.policy_forward(pop, H, states, gidx).cpu().numpy().reshape(n, S, 5, 2)
off = np.rint(raw.astype(np.float64) * 5.0)
ask, bid, bmax, smin = (np.asarray(tr[k])[idx] for k in (3, 4, 5, 6))
qa = ask[None, :, None] + off[..., 0] * 0.001
qb = bid[None, :, None] - off[..., 1] * 0.001
inv = invs[None, None, :]
fb = (inv < 2) & (qb >= smin[None, :, None])
fs = (inv > -2) & (qa <= bmax[None, :, None])
succ = inv + fb.astype(int) - fs.astype(int)
inj = np.array([[len(set(succ[i, t])) == 5 for t in range(S)] for i in range(n)])
score2 = inj.sum(1)
r2 = np.corrcoef(score2, slots)[0, 1]
t4, f4 = timeit(np.argsort(-score2, kind="stable"))
assert torch.equal(f0[0], f4[0])
print(f"predictor 2 corr(injective sampled ticks, slots) {r2:.2f}; ordered by it {t4:.1f} us")
