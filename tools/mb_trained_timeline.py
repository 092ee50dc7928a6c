"""Diagnostic: frontier-kernel wave timeline on GA-TRAINED populations (the state
bench.py times), stamped library (tools/build_stamps.sh).

Trains BASELINE config 3 (bench.make_engine, the bench's seeds) for G
generations, materializes the population of generation G with sgmm_ga_ask
(as tests/test_gpu_trained_state.py) and runs its 2560 training episodes
through the frontier kernel; prints per-wave durations / slots and the
per-SIMD picture (like mb_frontier_timeline.py).
    python tools/mb_trained_timeline.py [G=15] [config=3]"""
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
from sgmm_amd.drl_engine import ADV_GENOME
from sgmm_amd.model import genome_size

G_TRAIN = int(sys.argv[1]) if len(sys.argv) > 1 else 15
CONFIG = int(sys.argv[2]) if len(sys.argv) > 2 else 3
PHASE = bool(os.environ.get("PHASE"))
L = _lib.load()
L.sgmm_debug_frontier_tstamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
if not PHASE:
    L.sgmm_debug_frontier_thwid.argtypes = [ctypes.c_void_p, ctypes.c_int]
DEV = torch.device("cuda")
spec = dict(bench.CONFIGS[CONFIG])
P, H, T = spec["P"], spec["H"], spec["T"]
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
seg = ticks.segments[ticks.add(tr[0], st[0])]
ticks.to(DEV)
n = K * P
eps = sg.EpisodeBatch(np.arange(n), np.full(n, seg[0]), np.full(n, T), np.repeat(np.arange(K), P))
if os.environ.get("N_EPS"):  # N_EPS=64: 64 lone walks of population 0 (each alone on its SIMD; PHASE stamps rows = episodes)
    n = int(os.environ["N_EPS"])
    eps = sg.EpisodeBatch(np.arange(n), np.full(n, seg[0]), np.full(n, T), np.zeros(n))
    _lib.plan_set(policy_path="frontier", groups=1, min_eps=1)
if os.environ.get("ORDER"):  # population order of the walks (the first ones are whole walks), e.g. ORDER=1,4,0,2,3
    eps.order = np.concatenate([np.arange(k * P, (k + 1) * P) for k in map(int, os.environ["ORDER"].split(","))]
                               ).astype(np.int32)
eps = eps.to(DEV)
params = sg.params_tensor([sg.EnvConfig(phi=phi, tick_size=tick) for phi, tick, _ in spec["pops"]], DEV)
eng2 = sg.RolloutEngine(DEV)
for _ in range(3):
    eng2.fitness(ticks, eps, params, pop, H)
torch.cuda.synchronize()
if os.environ.get("SCAN"):
    # the path scan of the same launch (SGMM_STAMP slots, as tools/mb_scan3_stamps.py)
    L.sgmm_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    g_ = np.zeros((n, 16), np.uint64)
    L.sgmm_debug_stamps(g_.ctypes.data, n)
    g_ = g_.astype(np.int64)
    tot = (g_[:, 3] - g_[:, 0]).astype(float)
    print(f"scan, trained {G_TRAIN} generations: entry->end cycles p10 {np.percentile(tot, 10):.0f} med "
          f"{np.median(tot):.0f} p90 {np.percentile(tot, 90):.0f} p99 {np.percentile(tot, 99):.0f} max {tot.max():.0f}; "
          f"span {(g_[:, 3].max() - g_[:, 0].min()):.0f}")
    ga, sm, it, fb = g_[:, 11], g_[:, 12], g_[:, 13], g_[:, 14]
    pa, pb, wk = g_[:, 8] - g_[:, 2], g_[:, 9] - g_[:, 8], g_[:, 10] - g_[:, 9]
    print(f"  the last window (med / p90 cycles): phase a {np.median(pa):.0f}/{np.percentile(pa, 90):.0f}, phase b "
          f"{np.median(pb):.0f}/{np.percentile(pb, 90):.0f}, walk {np.median(wk):.0f}/{np.percentile(wk, 90):.0f}")
    print(f"  per episode: chunk starts med {np.median(g_[:, 1] - g_[:, 0]):.0f}, gather med {np.median(ga):.0f}, "
          f"exact sum med {np.median(sm):.0f}, walk iterations med {np.median(it):.0f}, fallback blocks med "
          f"{np.median(fb):.0f}")
    why = g_[:, 6].astype(np.uint64)
    nf, nb, ne = (why & 0xFFFFF).astype(float), ((why >> 20) & 0xFFFFF).astype(float), (why >> 40).astype(float)
    print(f"  blocks without a prediction per episode (med / p90): no binade {np.median(nf):.0f}/{np.percentile(nf, 90):.0f}, "
          f"bad step {np.median(nb):.0f}/{np.percentile(nb, 90):.0f}, binade edge {np.median(ne):.0f}/"
          f"{np.percentile(ne, 90):.0f}; zero blocks {np.median(g_[:, 7]):.0f}")
    t4, t5 = g_[:, 4], g_[:, 5]
    m_ = (t5 > t4) & (t4 > 0)
    if m_.any():
        print("  tell in the last arriver per population (e, cycles, end after the scan's first entry):",
              [(int(e), int(t5[e] - t4[e]), int(t5[e] - g_[:, 0].min())) for e in np.where(m_)[0][:8]],
              f"; the scan's last episode ends {int((g_[:, 3] * (g_[:, 3] > 0)).max() - g_[:, 0].min())}")
    o = np.argsort(tot)[::-1]
    print("  slowest (e, entry->end, gather, sum, iters, fallbacks):",
          [(int(e), int(tot[e]), int(ga[e]), int(sm[e]), int(it[e]), int(fb[e])) for e in o[:10]])
    for q in (50, 90, 99):
        m_ = tot >= np.percentile(tot, q)
        print(f"  >= p{q}: fallbacks {fb[m_].mean():.1f} iters {it[m_].mean():.1f} sum {sm[m_].mean():.0f} "
              f"gather {ga[m_].mean():.0f}")
    sys.exit(0)
h = np.zeros((n, 8), np.uint64)
L.sgmm_debug_frontier_tstamps(h.ctypes.data, n)
if PHASE:
    x = h.astype(np.float64)
    med = lambda a: float(np.median(a))
    CL = max(4, ((T + 63) // 64 + 3) // 4 * 4)
    print(f"trained {G_TRAIN} generations; waves {n}; chunk {CL} ticks")
    print(f"  cycles/wave {med(x[:, 0]):9.0f} wall {med(x[:, 7]) / 100:8.1f} us slots/wave {med(x[:, 3]):.0f}"
          f" cycles/slot {med(x[:, 0] / np.maximum(x[:, 3], 1)):.0f}")
    for k, lab in ((1, "L1+L2 issue"), (2, "L2 drain+tr+L3"), (4, "FPT+stores"), (5, "tick head"), (6, "tick tail")):
        print(f"  {lab:15s} {med(x[:, k]):9.0f} cyc/wave = {med(x[:, k]) / med(x[:, 0]) * 100:5.1f} %"
              f"  per slot {med(x[:, k] / np.maximum(x[:, 3], 1)):6.0f}")
    sys.exit(0)
# stamp rows: episode e's chunk group g at e + 16384 g (split episodes have two)
h = np.zeros((32768, 8), np.uint64)
L.sgmm_debug_frontier_tstamps(h.ctypes.data, 32768)
hw = np.zeros((32768, 2), np.uint32)
L.sgmm_debug_frontier_thwid(hw.ctypes.data, 32768)
rows = np.nonzero(h[:, 1])[0]
h, hw = h[rows], hw[rows]
n = len(rows)
t0 = h[:, 0].astype(np.int64)
t1 = h[:, 1].astype(np.int64)
base = t0.min()
s0, e_ = (t0 - base) * 10, (t1 - base) * 10  # ns
dur = e_ - s0
simd = (hw[:, 0] >> 4) & 3
cu = (hw[:, 0] >> 8) & 15
se = (hw[:, 0] >> 13) & 7
xcc = hw[:, 1] & 7
sid = ((xcc * 8 + se) * 16 + cu) * 4 + simd
sl = h[:, 2].astype(float)
print(f"trained {G_TRAIN} generations; waves {n}; kernel span {e_.max() / 1e3:.1f} us")
print(f"  duration med {np.median(dur) / 1e3:.1f} us p10 {np.percentile(dur, 10) / 1e3:.1f} "
      f"p90 {np.percentile(dur, 90) / 1e3:.1f} max {dur.max() / 1e3:.1f}")
print("  slots/wave percentiles 50/90/99/max:", [float(np.percentile(sl, p)) for p in (50, 90, 99)], float(sl.max()),
      f" total {sl.sum():.0f}")
u, inv = np.unique(sid, return_inverse=True)
cnt = np.bincount(inv)
last = np.zeros(len(u))
np.maximum.at(last, inv, e_)
grid = np.linspace(0, e_.max(), 40)
act = [(np.sum((s0 <= t) & (e_ > t))) for t in grid]
print("  resident waves over time (/1024 SIMDs):", [round(float(a) / 1024, 2) for a in act[::4]])
simd_slots = np.bincount(inv, weights=sl)
A = np.vstack([simd_slots, np.ones_like(simd_slots)]).T
coef, *_ = np.linalg.lstsq(A, last / 1e3, rcond=None)
print(f"  per-SIMD slots: mean {simd_slots.mean():.0f} max {simd_slots.max():.0f}; last end ~ {coef[0]:.3f} us/slot "
      f"+ {coef[1]:.1f} us, corr {np.corrcoef(simd_slots, last)[0, 1]:.2f}; SIMD last end med "
      f"{np.median(last) / 1e3:.1f} p90 {np.percentile(last, 90) / 1e3:.1f} max {last.max() / 1e3:.1f}")
for c in np.unique(cnt):
    m = cnt == c
    print(f"  SIMDs with {c} waves: {m.sum():4d}; last end med {np.median(last[m]) / 1e3:.1f} us max "
          f"{last[m].max() / 1e3:.1f}")
top = np.argsort(-e_)[:8]
print("  last-ending waves (end us, dur us, slots, waves on SIMD, SIMD slots):",
      [(round(e_[w] / 1e3, 1), round(dur[w] / 1e3, 1), int(sl[w]), int(cnt[inv[w]]), int(simd_slots[inv[w]]))
       for w in top])
print(f"  corr(slots, duration) {np.corrcoef(sl, dur)[0, 1]:.2f}; duration per slot of the 1% heaviest walks "
      f"{np.median(dur[sl >= np.percentile(sl, 99)] / sl[sl >= np.percentile(sl, 99)]) / 1e3:.2f} us")
# dispatch placement: do consecutive runs of 1024 blocks land one per SIMD?
for lo in range(0, n, 1024):
    hi = min(n, lo + 1024)
    su = np.unique(sid[lo:hi])
    print(f"  blocks {lo}-{hi - 1}: {len(su)} distinct SIMDs, {len(np.unique(sid[lo:hi] // 4))} distinct CUs")
order = np.argsort(s0, kind="stable")
print("  first 16 blocks: (XCD, SE, CU, SIMD)", [(int(xcc[b]), int(se[b]), int(cu[b]), int(simd[b])) for b in range(16)])
# early slot counts (slots in the first 8 / 16 ticks) as heaviness probes
s8 = h[:, 6].astype(float)
s16 = h[:, 7].astype(float)
whole = sl > 60  # whole walks (split halves have ~half the ticks)
for name, pr in (("s8", s8), ("s16", s16)):
    x, y = pr[whole], sl[whole]
    top = y >= np.percentile(y, 95)
    print(f"  {name}: percentiles 50/90/95/99 {[float(np.percentile(x, q)) for q in (50, 90, 95, 99)]}; corr with total "
          f"{np.corrcoef(x, y)[0, 1]:.2f}; top-5% walks' {name} med {np.median(x[top]):.0f} min {x[top].min():.0f}")
    for thr in np.percentile(x, [80, 90, 95]):
        sel = x >= thr
        print(f"    {name} >= {thr:.0f}: selects {sel.sum()} walks, catches {np.sum(sel & top)} of {top.sum()} top-5%;"
              f" their total slots med {np.median(y[sel]):.0f}")
# per population (episode e belongs to population e // P): the walks' slots and durations,
# and the episodes' total slots over their chunk groups
ep_of = rows % 16384
grp_of = rows // 16384
ep_slots = np.bincount(ep_of, weights=sl, minlength=K * P)
for k in range(K):
    m = (ep_of // P) == k
    es = ep_slots[k * P:(k + 1) * P]
    print(f"  population {k}: walks {m.sum()} (groups {sorted(set(grp_of[m].tolist()))}); walk slots med "
          f"{np.median(sl[m]):.0f} p99 {np.percentile(sl[m], 99):.0f}; walk duration med {np.median(dur[m]) / 1e3:.1f} "
          f"p99 {np.percentile(dur[m], 99) / 1e3:.1f} max {dur[m].max() / 1e3:.1f} us; episode slots med "
          f"{np.median(es):.0f} p99 {np.percentile(es, 99):.0f} max {es.max():.0f}")
