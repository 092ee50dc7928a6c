"""Parity of the state bench.py measures: GA-trained populations, not near-init ones.

bench.py times generations 5-24 of BASELINE config 3 (five lambda populations of
512, H=32, 4560 training ticks; best-validation generations, genomes generated
inside the rollout kernels from each population's device master, sigma and
Philox key).  Trained populations take different paths through the frontier
kernel than the near-init ones of test_gpu_configs.py (paths merge sooner; the
policy kernel goes from ~650 to ~480 us over the window), so here the bench's
own engine (bench.make_engine: rng="device", the same seeds, best validation)
is trained on the device for 24 generations, and then:

  1. the population generation 24 evaluates is materialized with sgmm_ga_ask
     (the rows the rollout kernels generate in registers), every training
     episode is rolled out through the C ABI's default policy path (the
     frontier kernel at 2560 episodes) and compared with the C oracle
     (oracle/sgmm_oracle.c, the reference's evaluate_individual,
     Env/drl_engine.py:9-67) -- fitness and trades bit-exact;
  2. the session then runs generation 24 itself (asked in-kernel, tell in the
     scan's tail): its history row -- best training fitness, its trades and
     index, the np.argmax of drl_engine.py:119-125 -- must equal the argmax of
     the materialized evaluation, which ties the benchmarked in-kernel path to
     the pinned one.

The same for BASELINE config 4's shape (256 market makers + 256 adversaries,
paired i <-> i, drl_engine.py:104-115) with trained adversaries, and for BASELINE
config 5 (two assets x 4096, tick sizes 0.001 and 0.01) whole and as the per-rank
shards of its 8- and 16-GPU runs (`bench.py --shard-of 8 / 16`: 2 x 512 episodes
in two chunk groups, 2 x 256 in four groups with two waves per walk) -- the launch
plans the strong-scaled runs take, on the populations they would train.  The
frontier spill (k_frontier_spill) is pinned the same way on config 3's trained
state, every walk forced to spill.
"""
import os

import numpy as np
import pytest
import torch

from conftest import has_gpu

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not has_gpu(), reason="needs a HIP device")]

DEV = torch.device("cuda:0")
THREADS = max(1, min(16, os.cpu_count() or 1))


def _pin_trained(sgmm, oracle, tmp_path, config, gens, shard_of=1, plan=None):
    import bench
    from sgmm_amd import _lib
    from sgmm_amd.drl_engine import ADV_GENOME, HIST_DTYPE
    from sgmm_amd.model import genome_size

    spec = dict(bench.CONFIGS[config])
    P, H, T = spec["P"], spec["H"], spec["T"]
    if shard_of > 1:  # one rank's shard of the strong-scaled run (bench.py --shard-of)
        from sgmm_amd.shard import shard_capacity
        P = shard_capacity(P, shard_of)
    K = len(spec["pops"])
    G = genome_size(H)
    data = bench.bundles(spec)
    tr = [data[a][0] for _, _, a in spec["pops"]]
    va = [data[a][1] for _, _, a in spec["pops"]]
    st = [data[a][2] for _, _, a in spec["pops"]]
    eng = bench.make_engine(sgmm, spec, P, str(tmp_path), None, True, "auto")
    sess = eng.session(tr, va, st, generations=gens + 1)
    assert sess.best_val and not sess.sharded
    sess.steps(0, gens)
    torch.cuda.synchronize()

    # 1. generation `gens`'s population, materialized
    L, s = sess.L, _lib.stream_ptr()
    pop = torch.empty((K * P, G), dtype=torch.float32, device=DEV)
    adv = torch.empty((K * P, ADV_GENOME), dtype=torch.float32, device=DEV) if spec["arl"] else None
    for k, e in enumerate(eng.engines):
        _lib.check(L.sgmm_ga_ask(_lib.ptr(sess.masters[k]), G, _lib.ptr(sess.states[k]), 0, e.seed, 0, P,
                                 _lib.ptr(pop[k * P:]), G, s), "sgmm_ga_ask")
        if adv is not None:
            _lib.check(L.sgmm_ga_ask(_lib.ptr(sess.masters_adv[k]), ADV_GENOME, _lib.ptr(sess.states[k]), 1,
                                     e.seed, 0, P, _lib.ptr(adv[k * P:]), ADV_GENOME, s), "sgmm_ga_ask(adv)")
    ticks = sgmm.TickStore()
    seg = {}
    for k in range(K):
        key = id(tr[k])
        if key not in seg:
            seg[key] = ticks.segments[ticks.add(tr[k], st[k])]
    ticks.to(DEV)
    offs = np.concatenate([np.full(P, seg[id(tr[k])][0]) for k in range(K)])
    lens = np.full(K * P, T)
    par = np.repeat(np.arange(K), P)
    ep_adv = np.arange(K * P) if adv is not None else None
    eps = sgmm.EpisodeBatch(np.arange(K * P), offs, lens, par, adv=ep_adv).to(DEV)
    params = sgmm.params_tensor([sgmm.EnvConfig(phi=phi, tick_size=tick) for phi, tick, _ in spec["pops"]], DEV)
    with _lib.plan(**(plan or {})):
        _lib.profile_read()
        _lib.profile_enable(True)
        try:
            fit, trd = sgmm.RolloutEngine(DEV).fitness(ticks, eps, params, pop, H, adv)
            kernels = _lib.profile_read()
        finally:
            _lib.profile_enable(False)
    torch.cuda.synchronize()
    if not spec["arl"]:
        assert "policy_frontier" in kernels, kernels  # the launch plan under test
    if plan and plan.get("spill"):
        assert "frontier_spill" in kernels, kernels
    got_f, got_t = fit.cpu().numpy(), trd.cpu().numpy()

    cols = [[], [], [], [], [], [], []]
    for key in seg:
        b = tr[[id(x) for x in tr].index(key)]
        s1n, s2n = oracle.normalize_signals(b[0], b[1], st[[id(x) for x in tr].index(key)])
        for c, a in zip(cols, (s1n, s2n) + tuple(b[2:])):
            c.append(a)
    tk = tuple(np.concatenate(c) for c in cols)
    plist = [oracle.params(phi=phi, tick=tick, fee=0.0) for phi, tick, _ in spec["pops"]]
    want_f, want_t = oracle.evaluate_batch(pop.cpu().numpy(), H, None if adv is None else adv.cpu().numpy(), tk,
                                           np.arange(K * P), ep_adv, offs, lens, par, plist, n_threads=THREADS)
    assert np.array_equal(got_t, want_t)
    assert np.array_equal(got_f, want_f)

    # 2. the session's own generation `gens` (asked inside the kernels)
    sess.steps(gens, 1)
    torch.cuda.synchronize()
    rows = sess.hist[:, gens].cpu().numpy().reshape(K, -1).view(HIST_DTYPE).reshape(K)
    f = got_f.reshape(K, P)
    for k in range(K):
        best = int(np.argmax(f[k]))
        assert int(rows[k]["best_idx"]) == best, k
        assert rows[k]["train_f"] == f[k, best], k
        assert int(rows[k]["train_trades"]) == int(got_t[k * P + best]), k
    sess.finish()
    return got_f, got_t


def test_config3_trained_populations_match_oracle(sgmm, oracle, tmp_path):
    f, t = _pin_trained(sgmm, oracle, tmp_path, config=3, gens=24)
    assert (t > 0).mean() > 0.5  # trading populations, not idle ones


def test_config4_trained_adversaries_match_oracle(sgmm, oracle, tmp_path):
    f, t = _pin_trained(sgmm, oracle, tmp_path, config=4, gens=24)
    assert (t > 0).mean() > 0.5


@pytest.mark.parametrize("shard_of", [1, 8, 16], ids=["whole", "shard_1_of_8", "shard_1_of_16"])
def test_config5_trained_populations_match_oracle(sgmm, oracle, tmp_path, shard_of):
    """Config 5 (2 x 4096, two assets) trained 20 generations on one GPU, and the
    per-rank shards of its 8- and 16-GPU runs trained as `bench.py --shard-of`
    trains them (2 x 512 episodes: two chunk groups per episode; 2 x 256: four
    groups, two waves per walk): bit-exact against the oracle."""
    f, t = _pin_trained(sgmm, oracle, tmp_path, config=5, gens=20, shard_of=shard_of)
    assert (t > 0).mean() > 0.5


def test_config3_trained_spill_match_oracle(sgmm, oracle, tmp_path):
    """The frontier spill on the benchmarked state: config 3 trained 24
    generations, every walk stopped at its first allowed tick (a 1 us deadline)
    and finished tick-parallel by k_frontier_spill -- bit-exact."""
    _pin_trained(sgmm, oracle, tmp_path, config=3, gens=24, plan={"spill": 1})


@pytest.mark.parametrize("T", [4560, 200], ids=["config3", "short_episodes"])
def test_config3_walk_reorder_same_results(sgmm, tmp_path, T):
    """The walk-order feedback (k_walk_reorder after each training launch of
    sgmm_generation_multi_best: the next launch walks the lightest populations whole)
    only schedules: 8 generations of config 3 with it and without it
    (walk_feedback=False: sgmm_populations::walk_order = NULL) give byte-identical
    history rows and masters; with it the session's walk order is a permutation of
    whole population blocks, and the episode batch's own order array (the ABI's
    read-only train_eps->order) is never written.  With 200-tick episodes the
    halves' second chunk group is empty (no slot count): the feedback scores only
    the groups that have chunks."""
    import bench
    spec = dict(bench.CONFIGS[3])
    spec["T"] = T
    P, K = spec["P"], len(spec["pops"])
    data = bench.bundles(spec)
    tr = [data[a][0] for _, _, a in spec["pops"]]
    va = [data[a][1] for _, _, a in spec["pops"]]
    st = [data[a][2] for _, _, a in spec["pops"]]
    out = {}
    for flag in (True, False):
        d = tmp_path / f"r{int(flag)}"
        d.mkdir()
        eng = bench.make_engine(sgmm, spec, P, str(d), None, True, "auto", walk_feedback=flag)
        sess = eng.session(tr, va, st, generations=9)
        sess.steps(0, 8)
        torch.cuda.synchronize()
        out[flag] = (sess.hist[:, :8].cpu().numpy().copy(), sess.masters.cpu().numpy().copy(),
                     sess.walk_order.cpu().numpy().copy(), sess.eps.dev["order"].cpu().numpy().copy())
        sess.finish()
    assert np.array_equal(out[True][0], out[False][0])
    assert np.array_equal(out[True][1], out[False][1])
    order = out[True][2]
    assert np.array_equal(np.sort(order), np.arange(K * P))
    for b in order.reshape(K, P):
        assert b[0] % P == 0 and np.array_equal(b, b[0] + np.arange(P))
    assert np.array_equal(out[False][2], np.arange(K * P))
    for flag in (True, False):  # the batch's order array is read-only
        assert np.array_equal(out[flag][3], np.arange(K * P))
    if T != 4560:
        return
    # the feedback does rewrite the walk order (eager generations, read after each;
    # which population is heaviest moves with training, so any one read may be the identity)
    d = tmp_path / "eager"
    d.mkdir()
    eng = bench.make_engine(sgmm, spec, P, str(d), None, False, "auto")
    sess = eng.session(tr, va, st, generations=4)
    seen = []
    for g in range(3):
        sess.step(g)
        torch.cuda.synchronize()
        seen.append(sess.walk_order.cpu().numpy().copy())
    sess.finish()
    assert any(not np.array_equal(o, np.arange(K * P)) for o in seen), "the feedback never reordered"
