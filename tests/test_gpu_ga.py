"""GPU tests of the device-resident GA loop (ask / tell / validation / sigma
decay) and of the drop-in DRLEngine against the reference's own training runs."""
import os

import numpy as np
import pytest
import torch

from conftest import has_gpu

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not has_gpu(), reason="needs a HIP device")]

DEV = torch.device("cuda:0")


def _state(sgmm, sigma=0.05, patience=15, decay=0.5):
    from sgmm_amd import _lib
    L = _lib.load()
    st = torch.zeros(80, dtype=torch.uint8, device=DEV)
    _lib.check(L.sgmm_ga_state_init(_lib.ptr(st), sigma, patience, decay, _lib.stream_ptr()), "init")
    return L, st


def _read_state(st):
    from sgmm_amd.drl_engine import STATE_DTYPE
    return st.cpu().numpy().view(STATE_DTYPE)[0]


def test_ask_deterministic_and_distributed(sgmm):
    from sgmm_amd import _lib
    L, st = _state(sgmm, sigma=0.5)
    G = 1250
    master = torch.randn(G, device=DEV)
    a = torch.empty((64, G), device=DEV)
    b = torch.empty((64, G), device=DEV)
    part = torch.empty((16, G), device=DEV)
    for out, i0, n in ((a, 0, 64), (b, 0, 64), (part, 40, 16)):
        _lib.check(L.sgmm_ga_ask(_lib.ptr(master), G, _lib.ptr(st), 0, 77, i0, n, _lib.ptr(out), G,
                                 _lib.stream_ptr()), "ask")
    assert torch.equal(a, b)                 # counter-based: reproducible
    assert torch.equal(a[40:56], part)       # any rank regenerates any individual
    z = ((a - master) / 0.5).double()
    assert abs(z.mean().item()) < 0.01 and abs(z.std().item() - 1.0) < 0.01
    adv = torch.empty((64, G), device=DEV)
    _lib.check(L.sgmm_ga_ask(_lib.ptr(master), G, _lib.ptr(st), 1, 77, 0, 64, _lib.ptr(adv), G,
                             _lib.stream_ptr()), "ask adv")
    assert not torch.equal(a, adv)           # independent adversary stream


def test_tell_argmax_semantics_and_regeneration(sgmm):
    from sgmm_amd import _lib
    G = 370
    cases = [
        ([0.5, 2.0, -1.0, 2.0], 1, 2),               # first max; adversary = first max of -f
        ([1.0, float("nan"), 3.0, float("nan")], 1, 1),  # np.argmax: first NaN wins
        ([-3.0] * 5, 0, 0),
    ]
    for fit, best, abest in cases:
        L, st = _state(sgmm, sigma=0.1)
        master = torch.randn(G, device=DEV)
        madv = torch.randn(1250, device=DEV)
        P = len(fit)
        pop = torch.empty((P, G), device=DEV)
        apop = torch.empty((P, 1250), device=DEV)
        _lib.check(L.sgmm_ga_ask(_lib.ptr(master), G, _lib.ptr(st), 0, 5, 0, P, _lib.ptr(pop), G,
                                 _lib.stream_ptr()), "ask")
        _lib.check(L.sgmm_ga_ask(_lib.ptr(madv), 1250, _lib.ptr(st), 1, 5, 0, P, _lib.ptr(apop), 1250,
                                 _lib.stream_ptr()), "ask")
        f = torch.tensor(fit, dtype=torch.float64, device=DEV)
        tr = torch.arange(P, dtype=torch.int32, device=DEV)
        hist = torch.zeros((4, 40), dtype=torch.uint8, device=DEV)
        _lib.check(L.sgmm_ga_tell(_lib.ptr(st), _lib.ptr(f), _lib.ptr(tr), P, _lib.ptr(master), None, G,
                                  _lib.ptr(madv), None, 1250, G, 1250, 5, _lib.ptr(hist), 4,
                                  _lib.stream_ptr()), "tell")
        s = _read_state(st)
        assert s["best_idx"] == best and s["adv_best_idx"] == abest, fit
        assert torch.equal(master, pop[best])      # regenerated in place == the asked genome
        assert torch.equal(madv, apop[abest])


def test_val_update_schedule(sgmm):
    """best_val / no_improve / sigma decay follow drl_engine.py:143-160."""
    from sgmm_amd import _lib
    from sgmm_amd.drl_engine import HIST_DTYPE
    L, st = _state(sgmm, sigma=0.05, patience=3, decay=0.5)
    G = 370
    master = torch.randn(G, device=DEV)
    best = torch.zeros(G, device=DEV)
    vals = [1.0, 0.5, 0.7, 0.9, 2.0, float("nan"), 1.0, 1.5, 1.9, 3.0]
    hist = torch.zeros((len(vals), 40), dtype=torch.uint8, device=DEV)
    model_best, noimp, sigma, flags = -np.inf, 0, 0.05, []
    for v in vals:
        vf = torch.tensor([v], dtype=torch.float64, device=DEV)
        vt = torch.tensor([7], dtype=torch.int32, device=DEV)
        _lib.check(L.sgmm_ga_val_update(_lib.ptr(st), _lib.ptr(vf), _lib.ptr(vt), 0, _lib.ptr(master),
                                        _lib.ptr(best), G, _lib.ptr(hist), len(vals), _lib.stream_ptr()),
                   "val")
        imp = v > model_best
        if imp:
            model_best, noimp = v, 0
        else:
            noimp += 1
        dec = noimp >= 3
        if dec:
            sigma *= 0.5
            noimp = 0
        flags.append(int(imp) | (int(dec) << 1))
    rows = hist.cpu().numpy().view(HIST_DTYPE).reshape(-1)
    assert list(rows["flags"]) == flags
    s = _read_state(st)
    assert s["sigma_mm"] == sigma and s["best_val"] == model_best and s["gen"] == len(vals)
    assert torch.equal(best, master)


@pytest.mark.parametrize("val_mode", ["best", "fused"])
@pytest.mark.parametrize("tag", ["drl", "arl"])
def test_drlengine_reproduces_reference_training(golden, sgmm, tmp_path, tag, val_mode):
    """rng='torch' + the same torch seed: identical history, final master and
    checkpoint to the reference DRLEngine.train (fixture g5, fork-faithful pool)."""
    d = golden("g5_ga.npz")
    arl = tag == "arl"
    tr = tuple(d[f"{tag}_train_{k}"] for k in ("s1", "s2", "mid", "ask", "bid", "buy_max", "sell_min"))
    va = tuple(d[f"{tag}_val_{k}"] for k in ("s1", "s2", "mid", "ask", "bid", "buy_max", "sell_min"))
    st = dict(zip(("s1_m", "s1_s", "s2_m", "s2_s"), (np.float32(x) for x in d[f"{tag}_stats"])))
    torch.manual_seed(int(d[f"{tag}_seed"]))
    eng = sgmm.DRLEngine(pop_size=6, sigma=0.05, phi=0.001, tick_size=0.001, use_arl=arl,
                         save_dir=str(tmp_path), rng="torch", verbose=False, val_mode=val_mode)
    pol, hist = eng.train(tr, va, st, generations=20, output_prefix="agent")
    for k in ("train_f", "val_f", "train_trades", "val_trades"):
        assert np.array_equal(np.array(hist[k], np.float64), d[f"{tag}_hist_{k}"]), k
    # torch's CPU normal sampler is vectorised per host ISA: on a different CPU
    # (the GPU box vs the fixture host) its draws can differ in the last ulp, so
    # genomes are compared to a few ulps; fitness/trades histories stay exact.
    w, ref = pol.get_weights().numpy(), d[f"{tag}_final_master"]
    err = np.abs(w.astype(np.float64) - ref)
    assert err.max() <= 1e-5, (err.max(), int((err > 0).sum()))
    ck = torch.load(os.path.join(tmp_path, "agent_best_val_0.001.pth"), weights_only=True)
    assert list(ck.keys()) == ["net.0.weight", "net.0.bias", "net.2.weight", "net.2.bias",
                               "net.4.weight", "net.4.bias"]
    ckw = torch.cat([ck[k].reshape(-1) for k in ck]).numpy()
    assert np.array_equal(ckw, w)  # the checkpoint holds exactly the returned policy
    assert np.abs(ckw.astype(np.float64) - d[f"{tag}_ckpt"]).max() <= 1e-5


def _bundles(seed=0, T=600, Tv=150):
    from sgmm_amd import synthetic
    tr = synthetic.bundle_510300(T, seed=seed)
    va = synthetic.bundle_510300(Tv, seed=seed + 1)
    return tr, va, synthetic.train_stats(tr)


@pytest.mark.parametrize("arl,P", [(False, 24), (True, 24), (False, 200), (False, 600), (True, 600)])
def test_device_rng_modes_agree(sgmm, tmp_path, arl, P):
    """graph replay == eager, fused validation == validate-the-best.  P=24:
    the 1024-thread scan's one-workgroup fused tail; P=200: 400 episodes, the
    512-thread scan (fused tail with P <= 512 threads); P=600: 1200 episodes,
    the 256-thread scan whose tail runs the general GA step."""
    tr, va, st = _bundles()
    res = []
    for use_graph, val_mode in ((True, "fused"), (False, "fused"), (False, "best"), (True, "best")):
        torch.manual_seed(0)  # the initial master is drawn from the torch generator
        eng = sgmm.DRLEngine(pop_size=P, phi=0.0005, tick_size=0.001, use_arl=arl,
                             save_dir=str(tmp_path / f"{use_graph}{val_mode}"), hidden_dim=16, rng="device",
                             seed=42, val_mode=val_mode, use_graph=use_graph, verbose=False, sync_every=7,
                             patience=4)
        pol, hist = eng.train(tr, va, st, generations=25)
        res.append((hist, pol.get_weights().numpy(), eng.mm_evolver.sigma))
    h0, w0, s0 = res[0]
    for h, w, s in res[1:]:
        for k in h0:
            assert np.array_equal(np.array(h[k], np.float64), np.array(h0[k], np.float64)), k
        assert np.array_equal(w, w0) and s == s0
    assert s0 < 0.05  # patience 4 over 25 generations decays sigma at least once


def test_device_modes_agree_with_nan_fitness(sgmm, tmp_path):
    """NaN training fitness (a NaN mid_next at ticks where only some
    individuals' quotes fill) follows np.argmax -- the first NaN wins -- in the
    fused in-scan GA step exactly as in the separate tell/val launches."""
    tr, va, st = _bundles(5)
    s1, s2, mid, ask, bid, bmax, smin = (a.copy() for a in tr)
    for j, t in enumerate(range(40, 600, 70)):
        mid[t] = np.nan
        smin[t] = np.nan                      # no buy fill at t
        bmax[t] = ask[t] + (j % 3 - 1) * 0.001  # a sell fill only for some offsets
    tr = (s1, s2, mid, ask, bid, bmax, smin)
    res = []
    for use_graph, val_mode in ((True, "fused"), (False, "best")):
        torch.manual_seed(3)
        eng = sgmm.DRLEngine(pop_size=24, sigma=0.2, phi=0.0005, tick_size=0.001, save_dir=str(tmp_path / val_mode),
                             hidden_dim=16, rng="device", seed=7, val_mode=val_mode, use_graph=use_graph,
                             verbose=False, sync_every=5, patience=4)
        pol, hist = eng.train(tr, va, st, generations=12)
        res.append((hist, pol.get_weights().numpy(), eng.mm_evolver.sigma))
    (h0, w0, s0), (h1, w1, s1_) = res
    assert np.isnan(np.array(h0["train_f"], np.float64)).any()  # the NaN path is exercised
    for k in h0:
        assert np.array_equal(np.array(h1[k], np.float64), np.array(h0[k], np.float64), equal_nan=True), k
    assert np.array_equal(w0, w1) and s0 == s1_


def test_device_ga_fitness_matches_reevaluation(sgmm, tmp_path):
    """history['train_f'] of each generation equals re-evaluating the master it
    produced, and the returned policy re-evaluates to the best validation reward."""
    from sgmm_amd.drl_engine import HIST_DTYPE
    tr, va, st = _bundles(3)
    eng = sgmm.DRLEngine(pop_size=32, phi=0.0005, tick_size=0.001, save_dir=str(tmp_path),
                         hidden_dim=16, seed=9, verbose=False)
    sess = eng.session(tr, va, st, generations=6)
    for g in range(6):
        sess.step(g)
        torch.cuda.synchronize()
        f, t = sgmm.evaluate_individual(sess.master.cpu(), None, tr, 0.0005, 0.001, 0.0, st)
        row = sess.hist[g].cpu().numpy().view(HIST_DTYPE)[0]
        assert f == row["train_f"] and t == row["train_trades"]
        fv, _ = sgmm.evaluate_individual(sess.master.cpu(), None, va, 0.0005, 0.001, 0.0, st)
        assert fv == row["val_f"]
    pol, hist = sess.finish()
    fv, _ = sgmm.evaluate_individual(pol.get_weights(), None, va, 0.0005, 0.001, 0.0, st)
    assert fv == max(hist["val_f"])


@pytest.mark.parametrize("arl", [False, True])
def test_ga_step_sharded_records_equal_contiguous(sgmm, arl):
    """sgmm_ga_step reading gathered per-rank records (shard_n, shard_stride)
    == reading contiguous population arrays."""
    from sgmm_amd import _lib
    from sgmm_amd.shard import FitnessRecords
    G, P, W = 370, 10, 3
    rng = np.random.default_rng(5)
    f = rng.normal(size=P); f[7] = f.max() + 1.0
    vf = rng.normal(size=P)
    t = rng.integers(0, 900, P).astype(np.int32)
    vt = rng.integers(0, 900, P).astype(np.int32)
    recs = [FitnessRecords(P, W, DEV) for _ in range(W)]
    gathered = torch.cat([r.rec for r in _fill(recs, f, t, vf, vt, P, W)])
    runs = []
    for sharded in (False, True):
        L, st = _state(sgmm, sigma=0.1)
        torch.manual_seed(1)
        master = torch.randn(G, device=DEV)
        madv = torch.randn(1250, device=DEV) if arl else None
        best = torch.zeros(G, device=DEV)
        hist = torch.zeros((2, 40), dtype=torch.uint8, device=DEV)
        if sharded:
            r = recs[0]
            r.gathered = gathered
            r.world = W
            args = r.step_args()
        else:
            cols = [torch.tensor(x, device=DEV) for x in (f, t, vf, vt)]
            args = tuple(_lib.ptr(c) for c in cols) + (P, 0, 0)
        _lib.check(L.sgmm_ga_step(_lib.ptr(st), *args, _lib.ptr(master), _lib.ptr(madv) if arl else None,
                                  _lib.ptr(best), G, 1250 if arl else 0, 9, _lib.ptr(hist), 2, None, None, 0, 0,
                                  _lib.stream_ptr()), "ga_step")
        torch.cuda.synchronize()
        runs.append((st.cpu(), master.cpu(), None if madv is None else madv.cpu(), best.cpu(), hist.cpu()))
    for a, b in zip(*runs):
        assert (a is None and b is None) or torch.equal(a, b)
    s = _read_state(runs[0][0])
    assert s["best_idx"] == 7 and s["adv_best_idx"] == int(np.argmax(-f))


def _fill(recs, f, t, vf, vt, P, W):
    from sgmm_amd.shard import shard_bounds
    for r, rec in enumerate(recs):
        i0, i1 = shard_bounds(P, r, W)
        n = i1 - i0
        rec.train[0][:n] = torch.tensor(f[i0:i1], device=DEV)
        rec.train[1][:n] = torch.tensor(t[i0:i1], device=DEV)
        rec.val[0][:n] = torch.tensor(vf[i0:i1], device=DEV)
        rec.val[1][:n] = torch.tensor(vt[i0:i1], device=DEV)
    return recs


def test_drlengine_two_ranks_equal_one(sgmm, tmp_path):
    """DRLEngine over 2 ranks (gloo exchange, both ranks on this GPU; the HIP
    graphs split around the all-gather) reproduces the single-process run."""
    import socket
    import torch.multiprocessing as mp
    import _shard_ranks as R
    P, gens = 24, 9
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    mp.spawn(R.train_rank, args=(2, port, P, gens, str(tmp_path)), nprocs=2, join=True)
    sg, tr, va, st, _ = R.workload(P, T=400, Tv=150)
    torch.manual_seed(0)
    eng = sg.DRLEngine(pop_size=P, phi=0.0005, tick_size=0.001, save_dir=str(tmp_path / "single"), hidden_dim=16,
                       rng="device", seed=11, verbose=False, sync_every=4, patience=3, dist=False)
    pol, hist = eng.train(tr, va, st, generations=gens)
    for r in range(2):
        o = np.load(tmp_path / f"t{r}.npz")
        for k in hist:
            assert np.array_equal(o[k], np.array(hist[k], np.float64)), (r, k)
        assert np.array_equal(o["w"], pol.get_weights().numpy())
        assert float(o["sigma"]) == eng.mm_evolver.sigma


def test_one_wave_tell_large_population(sgmm, tmp_path):
    """P=1100 with best validation: 1 100 training episodes take one-wave path
    scans, whose last workgroup runs the tell in one wave (tell_wave: records
    loaded 16 per lane at a time, two blocks here, DPP argmax).  Fused
    validation (2 200 episodes, the frontier kernel) gives the same run."""
    tr, va, st = _bundles(11, T=400, Tv=100)
    res = []
    for val_mode in ("best", "fused"):
        torch.manual_seed(4)
        eng = sgmm.DRLEngine(pop_size=1100, phi=0.0005, tick_size=0.001, save_dir=str(tmp_path / val_mode),
                             hidden_dim=16, rng="device", seed=21, val_mode=val_mode, verbose=False, sync_every=4,
                             patience=2)
        pol, hist = eng.train(tr, va, st, generations=8)
        res.append((hist, pol.get_weights().numpy(), eng.mm_evolver.sigma))
    (h0, w0, s0), (h1, w1, s1) = res
    for k in h0:
        assert np.array_equal(np.array(h0[k], np.float64), np.array(h1[k], np.float64), equal_nan=True), k
    assert np.array_equal(w0, w1) and s0 == s1
