"""GPU parity: every HIP entry point against the CPU oracle and the reference's
golden vectors.  Integer/state outputs (actions, inventories, fills, trades)
must be bit-exact; float64 cash/reward/fitness are bit-exact too (the kernels
keep the reference's operation order and sequential summation).
"""
import numpy as np
import pytest
import torch

from conftest import episodes_from_fixture, has_gpu, stats_dict

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not has_gpu(), reason="needs a HIP device")]

DEV = torch.device("cuda:0")


def _run_batch(sgmm, episodes, arl, trace=False):
    """Run a list of fixture-style episodes (same H) through the C ABI."""
    H = episodes[0]["H"]
    G = H * H + 7 * H + 2
    ticks = sgmm.TickStore()
    segs = []
    for ep in episodes:
        st = stats_dict(ep["stats"], ep["stats_nb"]) if "stats" in ep else ep["train_stats"]
        segs.append(ticks.add((ep["s1"], ep["s2"], ep["mid"], ep["ask"], ep["bid"], ep["buy_max"],
                               ep["sell_min"]), st))
    ticks.to(DEV)
    cfgs = [sgmm.EnvConfig(phi=ep["phi"], tick_size=ep["tick"], fee_rate=ep["fee"]) for ep in episodes]
    params = sgmm.params_tensor(cfgs, DEV)
    n = len(episodes)
    mm = torch.from_numpy(np.stack([ep["mm"][:G] for ep in episodes]).astype(np.float32)).to(DEV)
    adv = None
    adv_idx = None
    if arl:
        adv = torch.from_numpy(np.stack([ep["adv"] if ep["adv"] is not None else np.zeros(1250, np.float32)
                                         for ep in episodes])).to(DEV)
        adv_idx = np.array([i if ep["adv"] is not None else -1 for i, ep in enumerate(episodes)])
    eps = sgmm.EpisodeBatch(np.arange(n), [ticks.segments[s][0] for s in segs],
                            [ticks.segments[s][1] for s in segs], np.arange(n), adv=adv_idx).to(DEV)
    eng = sgmm.RolloutEngine(DEV)
    if trace:
        return eng.trace(ticks, eps, params, mm, H, adv), eps
    return eng.fitness(ticks, eps, params, mm, H, adv), eps


def _oracle_eval(oracle, ep, trace=False):
    p = oracle.params(phi=ep["phi"], tick=ep["tick"], fee=ep["fee"])
    return oracle.evaluate(ep["mm"], ep["H"], ep["adv"], ep["s1n"], ep["s2n"], ep["mid"], ep["ask"],
                           ep["bid"], ep["buy_max"], ep["sell_min"], p, trace=trace)


def _groups(eps):
    g = {}
    for ep in eps:
        g.setdefault((ep["H"], ep["adv"] is not None), []).append(ep)
    return g


@pytest.mark.parametrize("name", ["g2_synthetic.npz", "g3_adversary.npz"])
def test_fitness_matches_oracle(golden, sgmm, oracle, name):
    eps = list(episodes_from_fixture(golden(name)))
    for (H, arl), group in _groups(eps).items():
        (fit, trd), _ = _run_batch(sgmm, group, arl)
        fit, trd = fit.cpu().numpy(), trd.cpu().numpy()
        for i, ep in enumerate(group):
            f, t = _oracle_eval(oracle, ep)
            assert trd[i] == t, (name, ep["e"])
            assert fit[i] == f, (name, ep["e"], fit[i], f)


@pytest.mark.parametrize("name", ["g2_synthetic.npz", "g3_adversary.npz"])
def test_trace_matches_oracle(golden, sgmm, oracle, name):
    eps = list(episodes_from_fixture(golden(name)))
    for (H, arl), group in _groups(eps).items():
        (fit, trd, tr), eb = _run_batch(sgmm, group, arl, trace=True)
        tr = {k: v.cpu().numpy() for k, v in tr.items()}
        for i, ep in enumerate(group):
            f, t, want = _oracle_eval(oracle, ep, trace=True)
            sl = slice(int(eb.step_off[i]), int(eb.step_off[i]) + len(ep["mid"]))
            for k in want:
                assert np.array_equal(tr[k][sl], want[k]), (name, ep["e"], k)
            assert fit[i].item() == f and trd[i].item() == t


def test_g1_real_episode_actions(golden, sgmm):
    """ARL checkpoint on the recorded 510300 OOS episode (960 steps)."""
    d = golden("g1_arl_real.npz")
    ep = dict(H=32, mm=d["genome"], adv=None, s1=d["s1_pred"], s2=d["s2_pred"], mid=d["mid"],
              ask=d["ask"], bid=d["bid"], buy_max=d["buy_max"], sell_min=d["sell_min"], phi=0.0001,
              tick=0.001, fee=0.0, stats=d["stats"], stats_nb=True)
    (fit, trd, tr), _ = _run_batch(sgmm, [ep], False, trace=True)
    tr = {k: v.cpu().numpy() for k, v in tr.items()}
    for k in ("off_a", "off_b", "inventory", "fill_buy", "fill_sell", "cash", "reward"):
        assert np.array_equal(tr[k], d[k]), k
    assert fit[0].item() == float(d["fitness"]) and trd[0].item() == int(d["trades"])
    (fit2, trd2), _ = _run_batch(sgmm, [ep], False)
    assert fit2[0].item() == float(d["fitness"]) and trd2[0].item() == int(d["trades"])


def test_env_step_batch_edge_cases(golden, sgmm):
    d = golden("g4_ties.npz")
    n = len(d["mid"])
    env = sgmm.FTPEnvBatch(n, phi=d["phi"], tick_size=d["tick"], fee_rate=d["fee"], device=DEV)
    env.inventory.copy_(torch.from_numpy(d["inv_before"].astype(np.int32)))
    env.cash.copy_(torch.from_numpy(d["cash_before"]))
    act = np.stack([d["off_a"], d["off_b"]], 1)
    adv = np.stack([d["adv_a"], d["adv_b"]], 1)
    # rows without an adversary carry zero deltas: identical to adv_action=None
    r, info = env.step(act, d["mid"], d["ask"], d["bid"], d["buy_max"], d["sell_min"], adv_action=adv)
    assert np.array_equal(env.inventory.cpu().numpy(), d["inventory"])
    assert np.array_equal(env.cash.cpu().numpy(), d["cash"])
    assert np.array_equal(r.cpu().numpy(), d["reward"])
    assert np.array_equal(info["pnl_reward"].cpu().numpy(), d["pnl"])
    assert np.array_equal(info["inventory_reward"].cpu().numpy(), d["inv_reward"])
    assert np.array_equal(info["fee_paid"].cpu().numpy(), d["fee_paid"])
    assert np.array_equal(info["fill_buy"].cpu().numpy(), d["fill_buy"])
    assert np.array_equal(info["fill_sell"].cpu().numpy(), d["fill_sell"])


@pytest.mark.parametrize("H", [8, 16, 32, 64])
def test_policy_forward_bit_exact(sgmm, oracle, H):
    rng = np.random.default_rng(H)
    G = H * H + 7 * H + 2
    genomes = (rng.standard_normal((7, G)) * 0.4).astype(np.float32)
    n = 500
    idx = rng.integers(0, 7, n).astype(np.int32)
    states = np.stack([rng.standard_normal(n), rng.standard_normal(n),
                       rng.integers(-2, 3, n) / 2.0], 1).astype(np.float32)
    out = sgmm.policy_forward(torch.from_numpy(genomes).to(DEV), H, torch.from_numpy(states).to(DEV),
                              torch.from_numpy(idx).to(DEV)).cpu().numpy()
    want = np.stack([oracle.policy_forward(genomes[idx[i]], H, states[i]) for i in range(n)])
    assert np.array_equal(out, want)
    # and against the reference-shaped torch module within fp32 ordering slack
    pol = sgmm.TradingPolicy(hidden_dim=H)
    pol.set_weights(torch.from_numpy(genomes[0]))
    ref = pol(torch.from_numpy(states[idx == 0])).numpy()
    np.testing.assert_allclose(out[idx == 0], ref, rtol=1e-5, atol=1e-5)


def test_adversary_forward(sgmm, oracle):
    rng = np.random.default_rng(1)
    genomes = (rng.standard_normal((5, 1250)) * 3).astype(np.float32)
    n = 200
    idx = rng.integers(0, 5, n).astype(np.int32)
    states = np.stack([rng.integers(-2, 3, n) / 2.0, rng.integers(0, 2, n), rng.integers(0, 2, n)], 1).astype(np.float32)
    out = sgmm.adversary_forward(torch.from_numpy(genomes).to(DEV), torch.from_numpy(states).to(DEV),
                                 torch.from_numpy(idx).to(DEV)).cpu().numpy()
    want = np.stack([oracle.adversary_forward(genomes[idx[i]], states[i]) for i in range(n)])
    np.testing.assert_allclose(out, want, rtol=0, atol=2e-7)  # tanhf: ocml vs glibc, <= 1 ulp
    assert np.array_equal(np.rint(out), np.rint(want))


def _synthetic_batch(sgmm, P, T, H, seed, lengths=None, phi=0.001, nan_frac=0.0, sigma=0.3):
    from sgmm_amd import synthetic
    b = synthetic.bundle_510300(T, seed=seed, nan_frac=nan_frac)
    st = synthetic.train_stats(b)
    pop = synthetic.population(P, H, sigma=sigma, seed=seed + 1).numpy()
    lens = np.full(P, T) if lengths is None else np.asarray(lengths)
    eps = []
    for i in range(P):
        L = int(lens[i])
        s1n, s2n = sgmm.normalize_signals(b[0], b[1], st)
        eps.append(dict(H=H, mm=pop[i], adv=None, s1=b[0][:L], s2=b[1][:L], s1n=s1n[:L], s2n=s2n[:L],
                        mid=b[2][:L], ask=b[3][:L], bid=b[4][:L], buy_max=b[5][:L], sell_min=b[6][:L],
                        phi=phi, tick=0.001, fee=0.0, train_stats=st))
    return eps


def test_ragged_lengths_and_segment_boundaries(sgmm, oracle):
    """Lengths around the 64-tick chunk, 256-tick table block and 4096-tick
    summation segment boundaries, plus zero-length episodes."""
    lens = [0, 1, 63, 64, 65, 255, 256, 257, 4095, 4096, 4097, 9000]
    eps = _synthetic_batch(sgmm, len(lens), max(lens), 16, seed=11, lengths=lens)
    (fit, trd), _ = _run_batch(sgmm, eps, False)
    fit, trd = fit.cpu().numpy(), trd.cpu().numpy()
    for i, ep in enumerate(eps):
        f, t = _oracle_eval(oracle, ep)
        assert trd[i] == t and fit[i] == f, (lens[i], fit[i], f)
    assert fit[0] == -50.0 and trd[0] == 0  # empty episode: idle penalty only


def test_nan_bounds_and_h32_long(sgmm, oracle):
    eps = _synthetic_batch(sgmm, 6, 3600, 32, seed=21, nan_frac=0.03)
    (fit, trd), _ = _run_batch(sgmm, eps, False)
    for i, ep in enumerate(eps):
        f, t = _oracle_eval(oracle, ep)
        assert trd[i].item() == t and fit[i].item() == f


def test_bench_config_population(sgmm, oracle):
    """BASELINE config 2 shape (P=64, H=16, T=3600): every episode bit-exact."""
    from sgmm_amd import synthetic
    P, T, H = 64, 3600, 16
    b = synthetic.bundle_510300(T, seed=0)
    st = synthetic.train_stats(b)
    pop = synthetic.population(P, H, sigma=0.05, seed=1)
    fit, trd = sgmm.evaluate_population(pop, None, b, 0.0001, 0.001, 0.0, st)
    s1n, s2n = sgmm.normalize_signals(b[0], b[1], st)
    ticks = (s1n, s2n) + tuple(b[2:])
    want_f, want_t = oracle.evaluate_batch(pop.numpy(), H, None, ticks, np.arange(P), None,
                                           np.zeros(P), np.full(P, T), np.zeros(P),
                                           [oracle.params(phi=0.0001, tick=0.001)], n_threads=8)
    assert np.array_equal(trd, want_t)
    assert np.array_equal(fit, want_f)


@pytest.mark.parametrize("n_ep,caps,H,width", [(n, c, 16, None) for n in (400, 600, 1100) for c in ((2, -2), (3, -4))] +
                         [(n, (2, -2), h, None) for n in (600, 1100) for h in (8, 64)] +
                         [(400, (2, -2), 16, w) for w in (64, 512, 1024)] + [(1100, (3, -4), 16, 256)])
def test_many_episode_scan(sgmm, oracle, plan, n_ep, caps, H, width):
    """More than 256 / 512 episodes take the 4-wave / one-wave path scan (1024-tick
    windows; every width forced by the scan_threads plan override as well: 64,
    256, 512, 1024 threads; at H=16 400 episodes run the table, 600 and 1100 the
    frontier kernel; H=8 and H=64 have no frontier kernel, so 600 and 1100
    episodes take the table path into the one-wave scan): ragged lengths around
    their window boundaries, every episode bit-exact; with 5 inventory states
    (the default caps) and with 8 (i_max=3, i_min=-4: the NSM=8 scan
    instantiations)."""
    i_max, i_min = caps
    if width:
        plan(scan_threads=width)
    from sgmm_amd import synthetic
    T = 5000
    base = [0, 1, 17, 1023, 1024, 1025, 2047, 2048, 2049, 3600, 4096, 5000]
    lens = np.array([base[i % len(base)] if i < 96 else 700 + (37 * i) % 4300 for i in range(n_ep)], np.int64)
    P = len(lens)
    b = synthetic.bundle_510300(T, seed=3)
    st = synthetic.train_stats(b)
    pop = synthetic.population(P, H, sigma=0.2, seed=4)
    s1n, s2n = sgmm.normalize_signals(b[0], b[1], st)
    ticks = sgmm.TickStore()
    seg = ticks.add(b, st)
    ticks.to(DEV)
    params = sgmm.params_tensor([sgmm.EnvConfig(phi=0.0001, tick_size=0.001, i_max=i_max, i_min=i_min)], DEV)
    eb = sgmm.EpisodeBatch(np.arange(P), np.full(P, ticks.segments[seg][0]), lens, np.zeros(P),
                           inv_min=i_min, inv_max=i_max).to(DEV)
    fit, trd = sgmm.RolloutEngine(DEV).fitness(ticks, eb, params, pop.to(DEV), H)
    want_f, want_t = oracle.evaluate_batch(pop.numpy(), H, None, (s1n, s2n) + tuple(b[2:]), np.arange(P), None,
                                           np.zeros(P), lens, np.zeros(P),
                                           [oracle.params(phi=0.0001, tick=0.001, i_max=i_max, i_min=i_min)],
                                           n_threads=8)
    assert np.array_equal(trd.cpu().numpy(), want_t)
    assert np.array_equal(fit.cpu().numpy(), want_f)


def test_inventory_range_variants(sgmm, oracle):
    """Non-default caps (i_max=1, i_min=-3): 5 states, 0 not centred."""
    eps = _synthetic_batch(sgmm, 4, 700, 16, seed=31, sigma=0.5)
    ticks = sgmm.TickStore()
    segs = [ticks.add((e["s1"], e["s2"], e["mid"], e["ask"], e["bid"], e["buy_max"], e["sell_min"]),
                      e["train_stats"]) for e in eps]
    ticks.to(DEV)
    cfg = sgmm.EnvConfig(phi=0.002, tick_size=0.001, i_max=1, i_min=-3)
    params = sgmm.params_tensor([cfg], DEV)
    mm = torch.from_numpy(np.stack([e["mm"] for e in eps])).to(DEV)
    eb = sgmm.EpisodeBatch(np.arange(4), [ticks.segments[s][0] for s in segs], [700] * 4, np.zeros(4),
                           inv_min=-3, inv_max=1).to(DEV)
    fit, trd = sgmm.RolloutEngine(DEV).fitness(ticks, eb, params, mm, 16)
    for i, ep in enumerate(eps):
        p = oracle.params(phi=0.002, tick=0.001, i_max=1, i_min=-3)
        f, t = oracle.evaluate(ep["mm"], 16, None, ep["s1n"], ep["s2n"], ep["mid"], ep["ask"], ep["bid"],
                               ep["buy_max"], ep["sell_min"], p)
        assert trd[i].item() == t and fit[i].item() == f


def test_dropin_evaluate_individual(golden, sgmm):
    """The reference-signature entry point reproduces the reference's own fitness."""
    d = golden("g2_synthetic.npz")
    for ep in list(episodes_from_fixture(d))[:8]:
        st = stats_dict(ep["stats"], ep["stats_nb"])
        bundle = (ep["s1"], ep["s2"], ep["mid"], ep["ask"], ep["bid"], ep["buy_max"], ep["sell_min"])
        f, t = sgmm.evaluate_individual(torch.from_numpy(ep["mm"]), None if ep["adv"] is None else
                                        torch.from_numpy(ep["adv"]), bundle, ep["phi"], ep["tick"],
                                        ep["fee"], st, use_arl=ep["adv"] is not None)
        assert f == ep["fitness"] and t == ep["trades"]


def test_scan_ragged_lengths(golden, sgmm, oracle):
    """The path scan reproduces the oracle on the fixtures and on ragged
    lengths around the chunk / block / window boundaries."""
    eps = [e for e in episodes_from_fixture(golden("g2_synthetic.npz")) if e["adv"] is None]
    lens = [0, 1, 15, 16, 17, 63, 64, 65, 4095, 4096, 4097, 8193, 12000]
    eps += _synthetic_batch(sgmm, len(lens), max(lens), 16, seed=13, lengths=lens, sigma=0.3)
    for (H, arl), group in _groups(eps).items():
        (fit, trd), _ = _run_batch(sgmm, group, arl)
        for i, ep in enumerate(group):
            f, t = _oracle_eval(oracle, ep)
            assert trd[i].item() == t and fit[i].item() == f, (H, i)


@pytest.mark.parametrize("path", ["valu", "table", "table_v3", "frontier"])
def test_table_paths_agree(golden, sgmm, oracle, path, plan):
    """Every policy kernel -- the VALU table, the f32-MFMA tables (one state per
    wave for small launches, the v3 schedule forced by the table_sp=0 plan override;
    k_policy_table_mfma with the adversary and for H = 64) and the frontier
    kernel -- reproduces the oracle's canonical fma chains bit for bit (the MFMA
    k-order equals the chain)."""
    if path == "table_v3":
        plan(table_sp=0)
        path = "table"
    plan(policy_path=path)
    eps = list(episodes_from_fixture(golden("g2_synthetic.npz")))
    eps += _synthetic_batch(sgmm, 4, 1000, 32, seed=77, sigma=0.4)
    for (H, arl), group in _groups(eps).items():
        (fit, trd), _ = _run_batch(sgmm, group, arl)
        for i, ep in enumerate(group):
            f, t = _oracle_eval(oracle, ep)
            assert trd[i].item() == t and fit[i].item() == f, (path, H, arl, i)


@pytest.mark.parametrize("caps", [(0, 0), (1, -1), (2, -2), (3, -4)], ids=["nsi1", "nsi3", "nsi5", "nsi8"])
@pytest.mark.parametrize("H", [16, 32])
def test_state_parallel_table(sgmm, oracle, caps, H, plan):
    """The one-state-per-wave table (k_policy_table_sp, launches of at most 256
    chunks) and the v3 table agree bit for bit with each other and the oracle,
    for 1, 3, 5 and 8 inventory states and ragged lengths (partial last chunk,
    zero-length and one-tick episodes)."""
    from sgmm_amd import synthetic
    i_max, i_min = caps
    lens = np.array([0, 1, 63, 64, 65, 700, 912, 1000], np.int64)
    P, T = len(lens), int(lens.max())
    b = synthetic.bundle_510300(T, seed=5)
    st = synthetic.train_stats(b)
    pop = synthetic.population(P, H, sigma=0.3, seed=6)
    s1n, s2n = sgmm.normalize_signals(b[0], b[1], st)
    ticks = sgmm.TickStore()
    seg = ticks.add(b, st)
    ticks.to(DEV)
    params = sgmm.params_tensor([sgmm.EnvConfig(phi=0.0001, tick_size=0.001, i_max=i_max, i_min=i_min)], DEV)
    eb = sgmm.EpisodeBatch(np.arange(P), np.full(P, ticks.segments[seg][0]), lens, np.zeros(P),
                           inv_min=i_min, inv_max=i_max).to(DEV)
    plan(policy_path="table")
    got = {}
    for sp in ("1", "0"):
        plan(table_sp=int(sp))
        fit, trd = sgmm.RolloutEngine(DEV).fitness(ticks, eb, params, pop.to(DEV), H)
        got[sp] = (fit.cpu().numpy(), trd.cpu().numpy())
    want_f, want_t = oracle.evaluate_batch(pop.numpy(), H, None, (s1n, s2n) + tuple(b[2:]), np.arange(P), None,
                                           np.zeros(P), lens, np.zeros(P),
                                           [oracle.params(phi=0.0001, tick=0.001, i_max=i_max, i_min=i_min)],
                                           n_threads=8)
    for sp, (f, t) in got.items():
        assert np.array_equal(t, want_t), sp
        assert np.array_equal(f, want_f), sp


def _seq_sum(init, x):
    s = np.float64(init)
    for v in np.asarray(x, np.float64):
        s = s + v
    return s


def _sum_cases():
    rng = np.random.default_rng(11)
    tick = 2.0 ** -53
    env_like = np.where(rng.random(4320) < 0.4, 0.0,
                        np.where(rng.random(4320) < 0.5, -1e-4 * rng.integers(0, 3, 4320),
                                 rng.normal(4e-4, 1e-3, 4320)))
    ties = np.concatenate([[1.0], np.full(40, tick), [3 * tick, -tick, 2.0, 0.5 * tick], np.full(40, 3 * tick)])
    cancel = np.array([1.0, -1.0, 1e-300, -1e-300, 0.0, -0.0, 2.5, -2.5, 1e-3] * 30)
    subn = np.array([5e-324, 1e-310, -5e-324, 2.2250738585072014e-308, -1e-310] * 20)
    wide = rng.choice([-1.0, 1.0], 3000) * 2.0 ** rng.uniform(-60, 40, 3000)
    special = np.concatenate([rng.normal(0, 1, 100), [np.nan], rng.normal(0, 1, 50)])
    infs = np.concatenate([rng.normal(0, 1, 100), [np.inf], rng.normal(0, 1, 50), [-np.inf]])
    walk = rng.normal(1e-3, 2e-3, 100_000)
    boundary = np.array([0.5, 0.25, 0.25, -0.5, 0.125, 0.125, 0.25, 1.0, -2.0, 2.0 ** -30] * 50)
    return [("env_like", 0.0, env_like), ("ties", 0.0, ties), ("cancel", 0.0, cancel),
            ("subnormal", 0.0, subn), ("wide", 0.0, wide), ("nan", 0.0, special),
            ("inf", 0.0, infs), ("walk_100k", 0.0, walk), ("boundary", 0.0, boundary),
            ("init", 0.1, env_like[:1000]), ("neg_init", -3.0, env_like[:2000]),
            ("n0", 0.25, np.zeros(0)), ("n1", 0.0, np.array([0.3])), ("n15", 0.0, env_like[:15]),
            ("n16", 0.0, env_like[:16]), ("n17", 0.0, env_like[:17]), ("n4097", 0.0, env_like[:4097] * 1e3),
            # a binade edge crossed inside long runs (the walk's range check, not the prediction,
            # must stop the run), upwards, downwards and at negative sums
            ("edge_up", 1.0 - 3e-10, np.full(5000, 1e-13) + rng.normal(0, 1e-16, 5000)),
            ("edge_down", 2.0 + 2e-10, np.full(5000, -1e-13) + rng.normal(0, 1e-16, 5000)),
            ("edge_neg", -1.0 + 2e-10, np.full(5000, -1e-13)),
            ("zigzag", 0.0, np.tile([1e-3, -1e-3, 2e-3, -2e-3 + 1e-19], 1500)),
            ("exact_edges", 0.5 - 2.0 ** -40, np.full(4100, 2.0 ** -50)),
            # runs of exact zeros (an idle individual's rewards) are skipped whole by the walk
            ("idle", 0.0, np.zeros(4560)),
            ("idle_negzero", -0.0, np.zeros(100)),
            ("negzero_runs", -0.0, np.concatenate([-np.zeros(40), np.zeros(40), -np.zeros(40)])),
            ("zero_runs", 0.0, np.concatenate([np.zeros(2000), env_like[:500], -np.zeros(3000), env_like[:33],
                                               np.zeros(17), [1e-300], np.zeros(1000)])),
            ("zero_runs_inf", 0.0, np.concatenate([np.zeros(500), [np.inf], np.zeros(600), [1.0]])),
            ("zero_runs_init", 123.25, np.concatenate([np.zeros(1100), env_like[:300], np.zeros(5000)])),
            # streaks of blocks without a prediction (the walk adds a whole streak in one loop):
            # a mean-zero walk crossing zero, sums cancelling to tiny values, streaks cut by runs
            ("zero_mean_walk", 0.0, rng.normal(0, 1e-3, 20000)),
            ("crossings", 0.0, np.tile([1.0, -1.0 + 2.0 ** -40, 2.0 ** -60, -(2.0 ** -61)], 2500)),
            ("streaks_and_runs", 0.0, np.concatenate([np.tile([1e-3, -1e-3], 700), rng.normal(1e-3, 1e-4, 900),
                                                      np.tile([5e-4, -5e-4 - 1e-18], 1100), rng.normal(2e-3, 1e-4, 3000)]))]


@pytest.mark.parametrize("name,init,x", _sum_cases(), ids=[c[0] for c in _sum_cases()])
def test_ordered_sum_matches_sequential(sgmm, name, init, x):
    """The parallel exact episode sum (exact_sum_window, the path scan's sum)
    equals total += r in float64, bit for bit."""
    from sgmm_amd import _lib
    L = _lib.load()
    xd = torch.from_numpy(np.ascontiguousarray(x, np.float64)).to(DEV)
    out = torch.zeros(1, dtype=torch.float64, device=DEV)
    _lib.check(L.sgmm_ordered_sum(_lib.ptr(xd) if len(x) else None, len(x), float(init), _lib.ptr(out),
                                  _lib.stream_ptr()), "ordered_sum")
    got = out.cpu().numpy()[0]
    want = _seq_sum(init, x)
    if np.isnan(want):
        assert np.isnan(got)
    else:
        assert got.tobytes() == np.float64(want).tobytes(), (name, got, want)


@pytest.mark.parametrize("caps", [(0, 0), (0, -1), (1, 0)], ids=["1inv", "2inv_neg", "2inv_pos"])
def test_adversary_small_inventory_ranges(sgmm, oracle, caps):
    """Adversarial episodes with 1 or 2 inventory values (4 or 8 states of
    (inventory, previous fills)): the workspace takes the adversary layout
    (sgmm_rollout_workspace_bytes' explicit flag; a state count of 4 or 8
    alone reads as the no-adversary layout) and every episode is bit-exact
    against the oracle, 5000-tick episodes included."""
    i_max, i_min = caps
    from sgmm_amd import synthetic
    T, H, P = 5000, 16, 5
    b = synthetic.bundle_510300(T, seed=41)
    st = synthetic.train_stats(b)
    pop = synthetic.population(P, H, sigma=0.5, seed=42)
    rng = np.random.default_rng(43)
    adv = (rng.standard_normal((P, 1250)) * 2).astype(np.float32)
    lens = np.array([T, 1, 63, 777, 4096])
    s1n, s2n = sgmm.normalize_signals(b[0], b[1], st)
    ticks = sgmm.TickStore()
    seg = ticks.add(b, st)
    ticks.to(DEV)
    params = sgmm.params_tensor([sgmm.EnvConfig(phi=0.001, tick_size=0.001, i_max=i_max, i_min=i_min)], DEV)
    eb = sgmm.EpisodeBatch(np.arange(P), np.full(P, ticks.segments[seg][0]), lens, np.zeros(P),
                           adv=np.arange(P), inv_min=i_min, inv_max=i_max).to(DEV)
    eng = sgmm.RolloutEngine(DEV)
    nsi = i_max - i_min + 1
    assert eng.workspace_bytes(eb, True) == eng.L.sgmm_rollout_workspace_bytes(eb.n, eb.total_steps, nsi, 1)
    fit, trd = eng.fitness(ticks, eb, params, pop.to(DEV), H, torch.from_numpy(adv).to(DEV))
    fit, trd = fit.cpu().numpy(), trd.cpu().numpy()
    p = oracle.params(phi=0.001, tick=0.001, i_max=i_max, i_min=i_min)
    for i in range(P):
        L = int(lens[i])
        f, t = oracle.evaluate(pop[i].numpy(), H, adv[i], s1n[:L], s2n[:L], b[2][:L], b[3][:L], b[4][:L],
                               b[5][:L], b[6][:L], p)
        assert trd[i] == t and fit[i] == f, (caps, L, fit[i], f)


@pytest.mark.parametrize("seq", [0, 1], ids=["parallel_sum", "sequential_sum"])
@pytest.mark.parametrize("n_ep,H,arl", [(128, 16, False), (400, 16, False), (1100, 32, False), (64, 32, True),
                                          (1500, 32, True)],
                         ids=["16waves", "4waves", "1wave", "arl_16waves", "arl_4waves"])
def test_scan_sum_methods_agree(sgmm, oracle, plan, seq, n_ep, H, arl):
    """The path scans' two episode-sum methods -- the exact parallel binade method
    and the plain sequential chain (SGMM_PLAN_SEQ_SUM, chosen per launch by
    scan_seq_sum) -- give the oracle's bits at every scan width, with and without
    the adversary (whose scan sums 4096-tick segments), on ragged lengths and a
    wide population (sums near zero and crossing it)."""
    plan(seq_sum=seq)
    from sgmm_amd import synthetic
    lens = np.array([[0, 1, 17, 1023, 1024, 1025, 4095, 4096, 4097, 5000][i % 10] if i < 40 else 700 + (53 * i) % 4300
                     for i in range(n_ep)], np.int64)
    P = len(lens)
    T = int(lens.max())
    b = synthetic.bundle_510300(T, seed=11)
    st = synthetic.train_stats(b)
    pop = synthetic.population(P, H, sigma=0.6, seed=12)
    adv = synthetic.population(P, 32, sigma=0.3, seed=13) if arl else None
    ticks = sgmm.TickStore()
    seg = ticks.add(b, st)
    ticks.to(DEV)
    params = sgmm.params_tensor([sgmm.EnvConfig(phi=0.0005, tick_size=0.001)], DEV)
    eb = sgmm.EpisodeBatch(np.arange(P), np.full(P, ticks.segments[seg][0]), lens, np.zeros(P),
                           adv=np.arange(P) if arl else None).to(DEV)
    fit, trd = sgmm.RolloutEngine(DEV).fitness(ticks, eb, params, pop.to(DEV), H, adv.to(DEV) if arl else None)
    s1n, s2n = sgmm.normalize_signals(b[0], b[1], st)
    want_f, want_t = oracle.evaluate_batch(pop.numpy(), H, adv.numpy() if arl else None, (s1n, s2n) + tuple(b[2:]),
                                           np.arange(P), np.arange(P) if arl else None, np.zeros(P), lens,
                                           np.zeros(P), [oracle.params(phi=0.0005, tick=0.001)], n_threads=8)
    assert np.array_equal(trd.cpu().numpy(), want_t)
    assert np.array_equal(fit.cpu().numpy(), want_f)
