"""GPU tests of MultiDRLEngine: K GA populations (the lambda sweep of
BASELINE config 3, the per-asset runs of config 5) advanced in one launch pair
per generation must equal K independent DRLEngine.train runs bit for bit --
histories, final masters, sigma schedules and checkpoints
(agent_trainer.py:136-137 per phi, main.py:39-45; agent_trainer.py:168-173)."""
import os

import numpy as np
import pytest
import torch

from conftest import has_gpu

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not has_gpu(), reason="needs a HIP device")]


def _bundles():
    from sgmm_amd import synthetic
    a_tr = synthetic.bundle_510300(600, seed=10)
    a_va = synthetic.bundle_510300(150, seed=11)
    b_tr = synthetic.bundle_688981(520, seed=12)   # a second asset: other tick, other length
    b_va = synthetic.bundle_688981(170, seed=13)
    return (a_tr, a_va, synthetic.train_stats(a_tr)), (b_tr, b_va, synthetic.train_stats(b_tr))


# population k: (phi, tick, asset)
POPS = [(0.0001, 0.001, 0), (0.005, 0.001, 0), (0.01, 0.01, 1)]


def _engine(sgmm, k, P, arl, save_dir, H=16, val_mode="fused", use_graph=True):
    phi, tick, _ = POPS[k]
    torch.manual_seed(100 + k)  # the initial master (and adversary master) come from the torch generator
    return sgmm.DRLEngine(pop_size=P, phi=phi, tick_size=tick, use_arl=arl, save_dir=save_dir, hidden_dim=H,
                          rng="device", seed=1000 + 7 * k, val_mode=val_mode, sync_every=5, patience=3,
                          verbose=False, use_graph=use_graph)


@pytest.mark.parametrize("P,arl", [(24, False), (24, True), (300, False), (600, False)])
def test_multi_equals_independent_runs(sgmm, tmp_path, P, arl):
    """P=24: the tail's one-workgroup fused GA step; P=300/600 with 3 x 2P
    episodes: the 256-thread path scan, whose tail runs the general step."""
    assets = _bundles()
    gens = 12
    tr = [assets[a][0] for _, _, a in POPS]
    va = [assets[a][1] for _, _, a in POPS]
    st = [assets[a][2] for _, _, a in POPS]
    multi = sgmm.MultiDRLEngine([_engine(sgmm, k, P, arl, str(tmp_path / "multi")) for k in range(len(POPS))])
    assert multi.fused_path
    res = multi.train(tr, va, st, generations=gens)
    for k in range(len(POPS)):
        single = _engine(sgmm, k, P, arl, str(tmp_path / f"single{k}"))
        pol, hist = single.train(tr[k], va[k], st[k], generations=gens)
        mpol, mhist = res[k]
        for key in hist:
            assert np.array_equal(np.array(mhist[key], np.float64), np.array(hist[key], np.float64),
                                  equal_nan=True), (k, key)
        assert np.array_equal(mpol.get_weights().numpy(), pol.get_weights().numpy()), k
        me, se = multi.engines[k], single
        assert me.mm_evolver.sigma == se.mm_evolver.sigma, k
        if arl:
            assert torch.equal(me.adv_evolver.master_policy.get_weights(),
                               se.adv_evolver.master_policy.get_weights()), k
        name = f"agent_best_val_{POPS[k][0]}.pth"
        a = torch.load(os.path.join(tmp_path / "multi", name), weights_only=True)
        b = torch.load(os.path.join(tmp_path / f"single{k}", name), weights_only=True)
        assert all(torch.equal(a[x], b[x]) for x in b), k
    # the populations are live and distinct
    assert len({float(r[1]["train_f"][-1]) for r in res}) == len(POPS)


def test_multi_sweep_constructor_and_shared_bundle(sgmm, tmp_path):
    """MultiDRLEngine.sweep(phis) with one shared bundle == per-phi DRLEngines."""
    (tr, va, st), _ = _bundles()
    phis = [0.0001, 0.001, 0.005, 0.008, 0.01]
    torch.manual_seed(5)
    m = sgmm.MultiDRLEngine.sweep(phis, pop_size=16, tick_size=0.001, save_dir=str(tmp_path / "m"),
                                  hidden_dim=16, seeds=[11, 12, 13, 14, 15], sync_every=4, verbose=False)
    masters = [e.mm_evolver.master_policy.get_weights().clone() for e in m.engines]
    res = m.train(tr, va, st, generations=8)
    for k, phi in enumerate(phis):
        e = sgmm.DRLEngine(pop_size=16, phi=phi, tick_size=0.001, save_dir=str(tmp_path / f"s{k}"), hidden_dim=16,
                           seed=11 + k, sync_every=4, verbose=False)
        e.mm_evolver.master_policy.set_weights(masters[k])
        pol, hist = e.train(tr, va, st, generations=8)
        assert np.array_equal(np.array(res[k][1]["train_f"]), np.array(hist["train_f"])), phi
        assert np.array_equal(res[k][0].get_weights().numpy(), pol.get_weights().numpy()), phi


@pytest.mark.parametrize("P,arl,use_graph", [(24, False, True), (24, True, True), (300, False, False),
                                             (300, True, True), (400, False, True)])
def test_best_validation_equals_fused(sgmm, tmp_path, P, arl, use_graph):
    """val_mode="best" (sgmm_generation_multi_best: training launch with the
    tell in its tail, then ONE validation episode per population on the new
    master, drl_engine.py:127-138) == val_mode="fused" (every individual
    validated inside the training launch, the best's record picked): the
    validation of the best is the same episode on the same genome, so the
    histories, masters, sigma schedules and checkpoints agree bit for bit.
    P=400: 1 200 training episodes take one-wave path scans, whose tell runs in
    one wave (tell_wave); fused, 2 400 episodes run on the frontier kernel."""
    assets = _bundles()
    gens = 12
    tr = [assets[a][0] for _, _, a in POPS]
    va = [assets[a][1] for _, _, a in POPS]
    st = [assets[a][2] for _, _, a in POPS]
    out = {}
    for vm in ("fused", "best"):
        m = sgmm.MultiDRLEngine([_engine(sgmm, k, P, arl, str(tmp_path / vm), val_mode=vm, use_graph=use_graph)
                                 for k in range(len(POPS))])
        sess = m.session(tr, va, st, generations=gens)
        assert sess.best_val == (vm == "best")
        for g0 in range(0, gens, 5):
            n = min(5, gens - g0)
            sess.steps(g0, n)
            if n == 5:
                sess.flush(g0 + n)
        out[vm] = (sess.finish(), m)
    (rf, mf), (rb, mb) = out["fused"], out["best"]
    for k in range(len(POPS)):
        (pf, hf), (pb, hb) = rf[k], rb[k]
        for key in hf:
            assert np.array_equal(np.array(hf[key], np.float64), np.array(hb[key], np.float64), equal_nan=True), \
                (k, key)
        assert np.array_equal(pf.get_weights().numpy(), pb.get_weights().numpy()), k
        assert mf.engines[k].mm_evolver.sigma == mb.engines[k].mm_evolver.sigma, k
        if arl:
            assert torch.equal(mf.engines[k].adv_evolver.master_policy.get_weights(),
                               mb.engines[k].adv_evolver.master_policy.get_weights()), k
        name = f"agent_best_val_{POPS[k][0]}.pth"
        a = torch.load(os.path.join(tmp_path / "fused", name), weights_only=True)
        b = torch.load(os.path.join(tmp_path / "best", name), weights_only=True)
        assert all(torch.equal(a[x], b[x]) for x in b), k
    assert any(f < 0.05 for f in (e.mm_evolver.sigma for e in mb.engines))  # patience 3: a decay happened


@pytest.mark.parametrize("world,P,val_mode,arl,table_path", [
    (2, 25, "best", False, ""),
    (2, 25, "fused", True, ""),
    (3, 25, "best", True, ""),
    (3, 25, "fused", False, ""),
    (2, 25, "best", False, "frontier"),
], ids=["w2-best", "w2-fused-arl", "w3-best-arl", "w3-fused", "w2-best-frontier"])
def test_multi_sharded_ranks_equal_one_process(sgmm, tmp_path, world, P, val_mode, arl, table_path):
    """MultiDRLEngine over `world` ranks (gloo exchange, every rank on this GPU;
    P=25 does not divide by 2 or 3, so the last shard is short) equals the
    one-process MultiDRLEngine bit for bit: histories, final masters, adversary
    masters, sigma schedules and rank 0's checkpoints.  Each rank reads
    individual i of population k from the gathered records at
    (i / n) * K * record + k * stride + (i % n) * size, so shards i / n > 0 are
    read across ranks (sgmm_ga_tell_multi + sgmm_validate_multi with best
    validation, sgmm_ga_step_multi fused; Env/drl_engine.py:91-125)."""
    import socket

    import torch.multiprocessing as mp

    import _shard_ranks as R
    gens = 8
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    mp.spawn(R.multi_train_rank, args=(world, port, P, gens, str(tmp_path), val_mode, arl, table_path),
             nprocs=world, join=True)
    tr, va, st = R.multi_workload()
    from sgmm_amd import _lib
    with _lib.plan(policy_path=table_path or "auto"):
        single = R.multi_engines(sgmm, P, arl, str(tmp_path / "single"), val_mode, dist=False)
        want = R.multi_result(single, single.train(tr, va, st, generations=gens))
    for r in range(world):
        got = np.load(tmp_path / f"m{r}.npz")
        assert sorted(got.files) == sorted(want), r
        for key in want:
            assert np.array_equal(got[key], want[key], equal_nan=True), (r, key)
    for k, (phi, _, _) in enumerate(R.MULTI_POPS):
        name = f"agent_best_val_{phi}.pth"
        a = torch.load(os.path.join(tmp_path / "ck0", name), weights_only=True)
        b = torch.load(os.path.join(tmp_path / "single", name), weights_only=True)
        assert all(torch.equal(a[x], b[x]) for x in b), k
    # the populations trained and differ
    assert len({float(want[f"h{k}_train_f"][-1]) for k in range(len(R.MULTI_POPS))}) == len(R.MULTI_POPS)
