"""GPU parity of the frontier kernel (k_policy_frontier + the frontier path
scan): one wave per episode, lane = one of <= 64 chunks, only the inventory
states the chunk's paths occupy are evaluated, planes written once per tick
after the paths merge.  Every result must equal the CPU oracle bit for bit --
the same per-(tick, state) arithmetic as the table, a different schedule.
Reference: Env/drl_engine.py:9-67 (evaluate_individual), Env/market_env.py:22-67.
"""
import numpy as np
import pytest
import torch

from conftest import has_gpu

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not has_gpu(), reason="needs a HIP device")]

DEV = torch.device("cuda:0")


@pytest.fixture(params=[1, 2, 3, 4, 8, 16], ids=["1wave", "2waves", "3waves", "4waves", "8waves", "16waves"])
def frontier(plan, request):
    """The frontier kernel with the episodes cut into 1-16 chunk groups (one
    wave of 64 chunks each, chunks of frontier_len(T, groups) ticks; records
    e * 64 G + c, plane padding 256 G + 16 rows per episode)."""
    plan(policy_path="frontier", groups=request.param)


def _spilled_waves(roll, n, steps, groups, n_waves):
    """Waves of the last frontier launch that spilled: the wspill section of the
    workspace (sgmm_rollout.hip's layout: u64 cmaps | u64 ctr | u32 kinfo |
    u32 wslots | u32 wspill | planes, 256-byte aligned, records 64 G per episode)."""
    a256 = lambda x: (x + 255) & ~255
    nc, nfr = steps // 64 + n + 1, n * 64 * groups
    off = a256(max(nc, nfr) * 8) + a256(max(nc * 8, nfr * 32)) + a256(nfr * 4) + a256(n * 64 * 4)
    w = roll._ws[off:off + 4 * n_waves].cpu().numpy().view(np.uint32)
    return int((w != 0).sum())


def _run(sgmm, oracle, lens, H, seed, T=None, caps=(2, -2), nan_frac=0.0, sigma=0.2, phi=0.0005, fee=0.0,
         n_threads=8, arl=False, roll_out=None):
    from sgmm_amd import synthetic
    lens = np.asarray(lens, np.int64)
    P = len(lens)
    T = int(lens.max()) if T is None else T
    b = synthetic.bundle_510300(max(T, 1), seed=seed, nan_frac=nan_frac)
    st = synthetic.train_stats(b)
    pop = synthetic.population(P, H, sigma=sigma, seed=seed + 1)
    adv = synthetic.population(P, 32, sigma=0.05, seed=seed + 2) if arl else None
    i_max, i_min = caps
    ticks = sgmm.TickStore()
    seg = ticks.add(b, st)
    ticks.to(DEV)
    cfg = sgmm.EnvConfig(phi=phi, tick_size=0.001, fee_rate=fee, i_max=i_max, i_min=i_min)
    params = sgmm.params_tensor([cfg], DEV)
    eb = sgmm.EpisodeBatch(np.arange(P), np.full(P, ticks.segments[seg][0]), lens, np.zeros(P),
                           inv_min=i_min, inv_max=i_max).to(DEV)
    roll = sgmm.RolloutEngine(DEV)
    fit, trd = roll.fitness(ticks, eb, params, pop.to(DEV), H, adv.to(DEV) if arl else None)
    if roll_out is not None:
        roll_out.append(roll)
    s1n, s2n = sgmm.normalize_signals(b[0], b[1], st)
    want_f, want_t = oracle.evaluate_batch(pop.numpy(), H, adv.numpy() if arl else None,
                                           (s1n, s2n) + tuple(b[2:]), np.arange(P),
                                           np.arange(P) if arl else None,
                                           np.zeros(P), lens, np.zeros(P),
                                           [oracle.params(phi=phi, tick=0.001, fee=fee, i_max=i_max, i_min=i_min)],
                                           n_threads=n_threads)
    return fit.cpu().numpy(), trd.cpu().numpy(), want_f, want_t


@pytest.mark.parametrize("H", [16, 32])
def test_frontier_ragged_lengths(sgmm, oracle, frontier, H):
    """Chunk lengths from 4 ticks (T <= 256) up: lengths around 4 * 64, the
    chunk / window boundaries, a length not divisible by its chunk, 0 and 1."""
    lens = [0, 1, 2, 3, 4, 5, 63, 64, 65, 255, 256, 257, 258, 1000, 4095, 4096, 4097, 4560, 9001]
    fit, trd, wf, wt = _run(sgmm, oracle, lens, H, seed=41)
    assert np.array_equal(trd, wt)
    assert np.array_equal(fit, wf)
    assert fit[0] == -50.0 and trd[0] == 0


@pytest.mark.parametrize("caps", [(2, -2), (1, -1), (1, -3), (3, -4), (0, 0)],
                         ids=["5states", "3states", "offcentre", "8states", "1state"])
def test_frontier_inventory_ranges(sgmm, oracle, frontier, caps):
    """Caps other than +-2: 1, 3, 5 (inventory 0 off-centre) and 8 states."""
    fit, trd, wf, wt = _run(sgmm, oracle, [700, 2000, 3001, 64, 65], 16, seed=43, caps=caps, sigma=0.5)
    assert np.array_equal(trd, wt)
    assert np.array_equal(fit, wf)


def test_frontier_nan_bounds_fees_wide_population(sgmm, oracle, frontier):
    """NaN FPT bounds (no fill), fees, and a wide population (sigma 1: policies
    that quote far away, so paths merge late or never)."""
    fit, trd, wf, wt = _run(sgmm, oracle, [3600] * 12 + [720] * 12, 32, seed=45, nan_frac=0.05, sigma=1.0,
                            fee=3e-5)
    assert np.array_equal(trd, wt)
    assert np.array_equal(fit, wf)


@pytest.mark.parametrize("nw", ["", "1", "2", "4"], ids=["default", "1wave", "2waves", "4waves"])
def test_frontier_default_selection_many_episodes(sgmm, oracle, plan, nw):
    """From 512 episodes on the frontier kernel is the default: 2100 ragged
    episodes bit-exact against the oracle, whole or cut into 2 / 4 chunk
    groups."""
    if nw:
        plan(groups=int(nw))
    lens = 300 + (np.arange(2100) * 37) % 900
    fit, trd, wf, wt = _run(sgmm, oracle, lens, 16, seed=47, sigma=0.3)
    assert np.array_equal(trd, wt)
    assert np.array_equal(fit, wf)


def test_frontier_default_selection_config5_shard(sgmm, oracle):
    """One rank's shard of BASELINE config 5 on 8 GPUs: 2 x 512 individuals =
    1024 episodes of 3600 ticks, H = 32.  The measured table / frontier
    crossover lies between 512 and 1024 episodes (profiles/r03_c5_shard*), so
    the default selection runs the frontier kernel here; bit-exact against the
    oracle."""
    from sgmm_amd import _lib
    lens = 3600 - (np.arange(1024) % 5) * 4
    _lib.profile_read()
    _lib.profile_enable(True)
    try:
        fit, trd, wf, wt = _run(sgmm, oracle, lens, 32, seed=53, sigma=0.1)
        kernels = _lib.profile_read()
    finally:
        _lib.profile_enable(False)
    assert "policy_frontier" in kernels, kernels
    assert np.array_equal(trd, wt)
    assert np.array_equal(fit, wf)


@pytest.mark.parametrize("n", [512, 600], ids=["c5_16ranks", "600"])
def test_frontier_default_selection_small_shards(sgmm, oracle, n):
    """Config 5's shard on 16 GPUs (2 x 256 individuals = 512 episodes of 3600
    ticks, H = 32: 4 chunk groups per episode, 512-thread scan) and 600
    episodes (3 groups, one-wave scan) run the frontier kernel by default
    (profiles/r04_ab/r04m_*: 512 episodes 195-204 us frontier vs 255-263 us
    table); bit-exact against the oracle."""
    from sgmm_amd import _lib
    lens = 3600 - (np.arange(n) % 7) * 4
    _lib.profile_read()
    _lib.profile_enable(True)
    try:
        fit, trd, wf, wt = _run(sgmm, oracle, lens, 32, seed=57, sigma=0.1)
        kernels = _lib.profile_read()
    finally:
        _lib.profile_enable(False)
    assert "policy_frontier" in kernels, kernels
    assert np.array_equal(trd, wt)
    assert np.array_equal(fit, wf)


@pytest.mark.parametrize("spill", [1, 60, 150], ids=["spill_all", "spill60us", "spill150us"])
@pytest.mark.parametrize("groups,ls", [(1, 1), (2, 1), (4, 2)], ids=["whole", "halves", "quarters_ls2"])
@pytest.mark.parametrize("H", [16, 32])
def test_frontier_spill(sgmm, oracle, plan, spill, groups, ls, H):
    """The spill (k_frontier_spill): walks still running `spill` us after their start
    (1 = every walk, at its first allowed tick) stop with at most 64 ticks left in
    their chunks and the rest runs tick-parallel; the path scan reads the
    completed frontier layout.  Ragged lengths (short last chunks, chunks that had
    already ended at the stop, 16 / 32 / 64-tick remainders), 5 and 8 states, NaN
    bounds and fees, whole walks, halves and quarters with two waves per walk --
    bit-exact against the oracle, with walks actually spilled."""
    plan(policy_path="frontier", groups=groups, lane_split=ls, spill=spill)
    lens = [0, 1, 5, 63, 65, 257, 1000, 4097, 4560, 9001, 20000, 4560, 4560, 3600]
    for caps, nan, fee in (((2, -2), 0.0, 0.0), ((3, -4), 0.03, 3e-5)):
        rolls = []
        fit, trd, wf, wt = _run(sgmm, oracle, lens, H, seed=83, caps=caps, sigma=0.6, nan_frac=nan, fee=fee,
                                roll_out=rolls)
        assert np.array_equal(trd, wt)
        assert np.array_equal(fit, wf)
        n, steps = len(lens), int(np.sum(lens))
        nsp = _spilled_waves(rolls[0], n, steps, groups, n * groups * ls)
        if spill == 1:
            assert nsp >= n // 2, nsp
        else:
            assert nsp >= 0


@pytest.mark.parametrize("spill", [1, 100], ids=["spill_all", "spill100us"])
def test_frontier_spill_many_episodes_default_plan(sgmm, oracle, plan, spill):
    """The spill on the default launch plan of 2 100 ragged H = 32 episodes (the
    four-walk rule: whole walks and halves): bit-exact against the oracle."""
    plan(spill=spill)
    lens = 3000 + (np.arange(2100) * 37) % 1600
    fit, trd, wf, wt = _run(sgmm, oracle, lens, 32, seed=89, sigma=0.4)
    assert np.array_equal(trd, wt)
    assert np.array_equal(fit, wf)


def test_frontier_lifts_the_episode_length_cap(sgmm, oracle):
    """Episodes longer than the table's 131072-tick cap run on the frontier
    kernel (agent_trainer.py:74-77 concatenates days without a bound): a
    300 000-tick episode bit-exact."""
    fit, trd, wf, wt = _run(sgmm, oracle, [300000, 131073, 5], 32, seed=49, sigma=0.1)
    assert np.array_equal(trd, wt)
    assert np.array_equal(fit, wf)


@pytest.mark.parametrize("H", [16, 32])
def test_adversary_episodes_have_no_length_cap(sgmm, oracle, H):
    """The adversary path (drl_engine.py:43-48,97-100) has no episode cap
    either: its scan chains the chunk transducers segment by segment (4096
    ticks, the state entering each segment carried over), so a 300 000-tick
    ARL episode -- 74 segments -- and 131 073 / 4097 / 4096 / 5 / 0-tick ones
    are bit-exact against the oracle."""
    fit, trd, wf, wt = _run(sgmm, oracle, [300000, 131073, 4097, 4096, 5, 0], H, seed=53, sigma=0.1, arl=True)
    assert np.array_equal(trd, wt)
    assert np.array_equal(fit, wf)
    assert trd[0] > 1000


def test_frontier_training_equals_table(sgmm, tmp_path, plan):
    """DRLEngine (device RNG, fused validation) trains identically with the
    frontier kernel (whole episodes and 3 chunk groups) and the table:
    histories and final masters."""
    from sgmm_amd import synthetic
    tr = synthetic.bundle_510300(900, seed=51)
    va = synthetic.bundle_510300(200, seed=52)
    st = synthetic.train_stats(tr)
    out = {}
    for path in ("table", "frontier", "frontier3"):
        plan(policy_path="frontier" if path.startswith("frontier") else path, groups=3 if path == "frontier3" else 1)
        torch.manual_seed(7)
        eng = sgmm.DRLEngine(pop_size=40, phi=0.001, tick_size=0.001, save_dir=str(tmp_path / path), hidden_dim=32,
                             rng="device", seed=99, sync_every=4, verbose=False)
        pol, hist = eng.train(tr, va, st, generations=10)
        out[path] = (pol.get_weights().numpy(), hist)
    wa, ha = out["table"]
    for path in ("frontier", "frontier3"):
        wb, hb = out[path]
        for k in ha:
            assert np.array_equal(np.array(ha[k], np.float64), np.array(hb[k], np.float64), equal_nan=True), (path, k)
        assert np.array_equal(wa, wb), path


@pytest.mark.parametrize("val_mode", ["best", "fused"])
def test_frontier_multi_population_training(sgmm, tmp_path, plan, val_mode):
    """Three populations (two assets) trained on the frontier kernel (the
    scan's last workgroup per population runs its tell, or its whole GA step
    with fused validation) equal the table path bit for bit
    (Env/drl_engine.py:91-171)."""
    import _shard_ranks as R
    tr, va, st = R.multi_workload()
    out = {}
    for path in ("table", "frontier"):
        plan(policy_path=path)
        m = R.multi_engines(sgmm, 30, False, str(tmp_path / path), val_mode, dist=False)
        out[path] = R.multi_result(m, m.train(tr, va, st, generations=8))
    for key in out["table"]:
        assert np.array_equal(out["table"][key], out["frontier"][key], equal_nan=True), key


@pytest.mark.parametrize("nw", ["1", "2", "4", "8", "16"], ids=["1wave", "2waves", "4waves", "8waves", "16waves"])
def test_frontier_one_wave_scan_lengths(sgmm, oracle, plan, nw):
    """Above 512 episodes the path scan is one wave per episode (1024-tick
    windows of a 256-thread layout run by 64 lanes): chunk lengths from 4 to
    past 512 ticks, ragged last windows and chunks, both chunk groups of split
    episodes -- bit-exact against the oracle."""
    plan(policy_path="frontier", groups=int(nw))
    base = np.array([17, 255, 4560, 8191, 20001, 30003, 40000, 4097])
    n = 1100
    lens = base[np.arange(n) % len(base)] + (np.arange(n) // len(base)) % 7
    fit, trd, wf, wt = _run(sgmm, oracle, lens, 16, seed=51, sigma=0.3)
    assert np.array_equal(trd, wt)
    assert np.array_equal(fit, wf)


@pytest.mark.parametrize("ls,nw", [("2", "1"), ("2", "4"), ("4", "1"), ("4", "3")],
                         ids=["2waves_1group", "2waves_4groups", "4waves_1group", "4waves_3groups"])
@pytest.mark.parametrize("H", [16, 32])
def test_frontier_lane_split(sgmm, oracle, plan, ls, nw, H):
    """Lane split (k_policy_frontier<H, NSI, LS>): two or four waves per 64-chunk
    walk, each walking 32 or 16 of its chunks (the default from S/2 episodes
    down); ragged lengths, every group count, 5 and 8 states -- bit-exact."""
    plan(policy_path="frontier", lane_split=int(ls), groups=int(nw))
    lens = [0, 1, 5, 63, 65, 257, 1000, 4097, 4560, 9001]
    for caps in ((2, -2), (3, -4)):
        fit, trd, wf, wt = _run(sgmm, oracle, lens, H, seed=71, caps=caps, sigma=0.5)
        assert np.array_equal(trd, wt), caps
        assert np.array_equal(fit, wf), caps


@pytest.mark.parametrize("fused", [0, 1], ids=["separate_scan", "fused_scan"])
@pytest.mark.parametrize("groups", [1, 2, 3], ids=["whole", "halves", "thirds"])
@pytest.mark.parametrize("H", [16, 32])
def test_frontier_fused_scan(sgmm, oracle, plan, fused, groups, H):
    """The path scan fused into the frontier launch (k_policy_frontier<..., FS>):
    each walk sums its own chunk group; of an episode walked in halves, group 0
    hands the chain (sum, state, trades) on to group 1, or continues over group
    1's handed-over rows when group 1 finished first.  Against the separate scan
    launch and the oracle, bit for bit: empty and one-tick episodes (group 0
    stores the record without a walk), halves whose second group has no chunks,
    ragged lengths across the 512-tick windows; more than two groups keep the
    separate scan."""
    from sgmm_amd import _lib
    plan(policy_path="frontier", groups=groups, fused_scan=fused)
    lens = [0, 1, 5, 64, 257, 511, 512, 513, 4560, 0, 9001, 3600, 700, 2]
    _lib.profile_read()
    _lib.profile_enable(True)
    try:
        fit, trd, wf, wt = _run(sgmm, oracle, lens, H, seed=53, sigma=0.4)
        kinds = _lib.profile_read()
    finally:
        _lib.profile_enable(False)
    assert np.array_equal(trd, wt)
    assert np.array_equal(fit, wf)
    assert fit[0] == -50.0 and trd[0] == 0 and fit[9] == -50.0
    assert "policy_frontier" in kinds
    assert ("path_scan" in kinds) == (fused == 0 or groups > 2)


@pytest.mark.parametrize("seed", [61, 62, 63])
def test_frontier_fused_scan_handoff_both_ways(sgmm, oracle, plan, seed):
    """Halves of very different weight: wide policies (paths that rarely merge) and
    ragged lengths, 1 200 episodes whose two groups finish in either order -- group
    0 last (it continues over group 1's handed-over rows) or group 1 last (it
    continues group 0's chain); which order each episode takes is not observed
    here, only that every result is bit-exact."""
    plan(policy_path="frontier", groups=2, fused_scan=1)
    lens = 1000 + (np.arange(1200) * 53) % 3700
    fit, trd, wf, wt = _run(sgmm, oracle, lens, 32, seed=seed, sigma=1.0, nan_frac=0.02)
    assert np.array_equal(trd, wt)
    assert np.array_equal(fit, wf)


@pytest.mark.parametrize("lanes", [0, 2, 4], ids=["one_wave_scan", "lanes_scan_w2", "lanes_scan_w4"])
@pytest.mark.parametrize("groups", [1, 2, 4, 16], ids=["whole", "halves", "quarters", "16groups"])
def test_frontier_lanes_scan(sgmm, oracle, plan, lanes, groups):
    """The frontier path scan with 2 or 4 episodes per workgroup, their sequential chains
    in the lanes of one wave (k_path_scan_lanes), against the one-wave scan and the
    oracle: ragged lengths (the shorter episodes' windows padded with -0.0), empty
    and one-tick episodes, a batch that is not a multiple of 2 or 4, 1-16 chunk groups."""
    plan(policy_path="frontier", groups=groups, lanes_scan=lanes, fused_scan=0)
    lens = [0, 1, 5, 64, 257, 511, 512, 513, 4560, 0, 9001, 3600, 700, 2, 1023, 1024, 1025, 4096, 100, 7,
            300, 301, 302, 2049, 17, 4561, 0, 33, 8191, 250, 251, 3001, 999, 1000, 1001, 64, 65]
    fit, trd, wf, wt = _run(sgmm, oracle, lens, 32, seed=71, sigma=0.5)
    assert np.array_equal(trd, wt)
    assert np.array_equal(fit, wf)


@pytest.mark.parametrize("caps", [(3, -4), (1, -3), (0, 0)], ids=["8states", "offcentre", "1state"])
def test_frontier_lanes_scan_inventory_ranges(sgmm, oracle, plan, caps):
    """The lanes scan (k_path_scan_lanes<8> for 8 inventory states, <5> otherwise)
    with caps other than +-2, NaN FPT bounds and fees, ragged lengths."""
    plan(policy_path="frontier", groups=2, lanes_scan=1, fused_scan=0)
    lens = 200 + (np.arange(23) * 211) % 2500
    fit, trd, wf, wt = _run(sgmm, oracle, lens, 16, seed=73, caps=caps, sigma=0.6, nan_frac=0.03, fee=2e-5)
    assert np.array_equal(trd, wt)
    assert np.array_equal(fit, wf)
