"""GPU parity at BASELINE.json's full configuration sizes (configs 3-5; config 2
is test_gpu_parity.py::test_bench_config_population).  Every episode of each
configuration's rollout is compared with the C oracle (8-16 OpenMP threads):
fitness (float64) and trades bit-exact.

  config 3  P=512 x lambda in {0.0001, 0.001, 0.005, 0.008, 0.01}: 2560 episodes
            over one full trading day at event_step=1 (T=4560), H=32
  config 4  adversarial co-training shape: 256 MM + 256 adversary genomes paired
            i<->i (drl_engine.py:104-115), T=3600, H=32; half the adversaries
            scaled x50 so tanh saturates and the offsets move (the LUT path)
  config 5  two assets (510300: tick 0.001 around 3.49; 688981: tick 0.01 around
            45.00) x P=4096, T=3600, mixed tick sizes and phi in one launch --
            the whole 8-GPU population on one GPU, and one rank's 512/asset shard

Tick streams are synthetic (synthetic.py): the reference ships no LOB
data.  The reference tick/phi choices per asset follow agent_trainer.py:168-173.
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


def _run(sgmm, oracle, bundles, stats, pop, adv, ep_genome, ep_bundle, ep_adv, ep_param, cfgs, H):
    """Same episode batch through the C ABI and the oracle; returns both."""
    ticks = sgmm.TickStore()
    segs = [ticks.add(b, st) for b, st in zip(bundles, stats)]
    ticks.to(DEV)
    offs = np.array([ticks.segments[s][0] for s in segs])[ep_bundle]
    lens = np.array([ticks.segments[s][1] for s in segs])[ep_bundle]
    params = sgmm.params_tensor([sgmm.EnvConfig(**c) for c in cfgs], DEV)
    eps = sgmm.EpisodeBatch(ep_genome, offs, lens, ep_param, adv=ep_adv).to(DEV)
    mm = torch.from_numpy(pop).to(DEV)
    advt = torch.from_numpy(adv).to(DEV) if adv is not None else None
    fit, trd = sgmm.RolloutEngine(DEV).fitness(ticks, eps, params, mm, H, advt)
    torch.cuda.synchronize()
    # oracle over the same concatenated streams
    cols = [[], [], [], [], [], [], []]
    for b, st in zip(bundles, stats):
        s1n, s2n = oracle.normalize_signals(b[0], b[1], st)
        for c, a in zip(cols, (s1n, s2n) + tuple(b[2:])):
            c.append(a)
    tk = tuple(np.concatenate(c) for c in cols)
    plist = [oracle.params(phi=c["phi"], tick=c["tick_size"], fee=c.get("fee_rate", 0.0)) for c in cfgs]
    want_f, want_t = oracle.evaluate_batch(pop, H, adv, tk, ep_genome, ep_adv, offs, lens, ep_param,
                                           plist, n_threads=THREADS)
    return fit.cpu().numpy(), trd.cpu().numpy(), want_f, want_t


def test_config3_lambda_sweep_full_day(sgmm, oracle):
    from sgmm_amd import synthetic
    P, T, H = 512, 4560, 32
    lams = [0.0001, 0.001, 0.005, 0.008, 0.01]
    b = synthetic.bundle_510300(T, seed=30)
    st = synthetic.train_stats(b)
    pop = synthetic.population(P, H, sigma=0.05, seed=31).numpy()
    E = P * len(lams)
    ep_genome = np.tile(np.arange(P), len(lams))
    ep_param = np.repeat(np.arange(len(lams)), P)
    got_f, got_t, want_f, want_t = _run(sgmm, oracle, [b], [st], pop, None, ep_genome,
                                        np.zeros(E, int), None, ep_param,
                                        [dict(phi=l, tick_size=0.001) for l in lams], H)
    assert np.array_equal(got_t, want_t)
    assert np.array_equal(got_f, want_f)
    # the sweep is live: a larger lambda never raises a genome's fitness here
    # (same trajectory when inventory stays 0, lower reward otherwise)
    f = got_f.reshape(len(lams), P)
    assert (np.diff(f, axis=0) <= 0).mean() > 0.95


def test_config4_adversarial_pairs(sgmm, oracle):
    from sgmm_amd import synthetic
    P, T, H = 256, 3600, 32
    b = synthetic.bundle_510300(T, seed=40)
    st = synthetic.train_stats(b)
    pop = synthetic.population(P, H, sigma=0.05, seed=41).numpy()
    adv = synthetic.population(P, 32, sigma=0.05, seed=42).numpy()  # TradingPolicy-layout genomes
    adv[P // 2:] *= 50.0  # saturated adversaries: tanh -> +-1, offsets shift
    got_f, got_t, want_f, want_t = _run(sgmm, oracle, [b], [st], pop, adv, np.arange(P),
                                        np.zeros(P, int), np.arange(P), np.zeros(P, int),
                                        [dict(phi=0.0001, tick_size=0.001)], H)
    assert np.array_equal(got_t, want_t)
    assert np.array_equal(got_f, want_f)
    # the adversary matters: the same MM genomes without it score differently
    nf, nt, _, _ = _run(sgmm, oracle, [b], [st], pop[P // 2:], None, np.arange(P // 2),
                        np.zeros(P // 2, int), None, np.zeros(P // 2, int),
                        [dict(phi=0.0001, tick_size=0.001)], H)
    assert (nf != got_f[P // 2:]).mean() > 0.5


@pytest.mark.parametrize("shard", ["full", "rank_shard"])
def test_config5_multi_asset(sgmm, oracle, shard):
    from sgmm_amd import synthetic
    P, T, H = 4096, 3600, 32
    n = P if shard == "full" else P // 8  # one of 8 ranks: 512 per asset
    bundles = [synthetic.bundle_510300(T, seed=50), synthetic.bundle_688981(T, seed=51)]
    stats = [synthetic.train_stats(bb) for bb in bundles]
    pop = synthetic.population(2 * n, H, sigma=0.05, seed=52).numpy()  # one population per asset
    ep_genome = np.arange(2 * n)
    ep_bundle = np.repeat([0, 1], n)
    cfgs = [dict(phi=0.0001, tick_size=0.001), dict(phi=0.01, tick_size=0.01)]
    got_f, got_t, want_f, want_t = _run(sgmm, oracle, bundles, stats, pop, None, ep_genome, ep_bundle,
                                        None, ep_bundle, cfgs, H)
    assert np.array_equal(got_t, want_t)
    assert np.array_equal(got_f, want_f)
