"""Pins the CPU oracle to the reference's own outputs (golden fixtures).

CPU-only.  The oracle is the checker for every GPU parity test, so it must
itself reproduce what the imported reference produced (tests/golden/gen_golden.py).
"""
import numpy as np
import pytest

from conftest import agree_until_justified_divergence, episodes_from_fixture, stats_dict


def test_g1_real_arl_policy_and_env(golden, oracle):
    """ARL checkpoint on the recorded 510300 OOS episode: 960/960 actions,
    inventory/fills/cash/reward bit-exact (ipynb:856 fills = 1568 for ARL)."""
    d = golden("g1_arl_real.npz")
    p = oracle.params(phi=0.0001, tick=0.001, fee=0.0)
    fit, trades, tr = oracle.evaluate(d["genome"], 32, None, d["s1n"], d["s2n"], d["mid"], d["ask"],
                                      d["bid"], d["buy_max"], d["sell_min"], p, trace=True)
    assert np.array_equal(tr["off_a"], d["off_a"])
    assert np.array_equal(tr["off_b"], d["off_b"])
    assert np.array_equal(tr["inventory"], d["inventory"])
    assert np.array_equal(tr["fill_buy"], d["fill_buy"])
    assert np.array_equal(tr["fill_sell"], d["fill_sell"])
    assert np.array_equal(tr["cash"], d["cash"])
    assert np.array_equal(tr["reward"], d["reward"])
    assert fit == float(d["fitness"]) and trades == int(d["trades"])
    assert int(d["fill_buy"].sum() + d["fill_sell"].sum()) == 1568
    # raw outputs: canonical fma order vs torch/MKL order differ by a few ulp only
    np.testing.assert_allclose(tr["raw_a"], d["raw"][:, 0], rtol=0, atol=2e-6)
    np.testing.assert_allclose(tr["raw_b"], d["raw"][:, 1], rtol=0, atol=2e-6)


def test_g1_normalisation_matches_reference(golden, oracle):
    d = golden("g1_arl_real.npz")
    st = stats_dict(d["stats"], nb=True)
    a, b = oracle.normalize_signals(d["s1_pred"], d["s2_pred"], st)
    assert np.array_equal(a, d["s1n"]) and np.array_equal(b, d["s2n"])


@pytest.mark.parametrize("method", ["arl", "drl", "glft", "foic"])
def test_g1_env_replay_bit_exact(golden, oracle, method):
    d = golden("g1_env_replay.npz")
    g = {k.split("__", 1)[1]: v for k, v in d.items() if k.startswith(method + "__")}
    p = oracle.params(phi=0.0001, tick=0.001, fee=0.0)
    inv, cash = 0, 0.0
    for t in range(len(g["mid"])):
        inv, cash, r, pnl, ir, fee, fb, fs = oracle.env_step(
            p, inv, cash, g["off_a"][t], g["off_b"][t], None, g["mid"][t], g["ask"][t], g["bid"][t],
            g["buy_max"][t], g["sell_min"][t])
        assert inv == g["inventory"][t] and cash == g["cash"][t] and r == g["reward"][t]
        assert pnl == g["pnl"][t] and ir == g["inv_reward"][t] and fee == g["fee_paid"][t]
        assert fb == g["fill_buy"][t] and fs == g["fill_sell"][t]


def test_g4_fill_test_edge_cases(golden, oracle):
    """Decimal-grid ties (fp64 quote arithmetic decides), NaN bounds, caps, fees."""
    d = golden("g4_ties.npz")
    for t in range(len(d["mid"])):
        p = oracle.params(phi=float(d["phi"][t]), tick=float(d["tick"][t]), fee=float(d["fee"][t]))
        adv = (int(d["adv_a"][t]), int(d["adv_b"][t])) if d["has_adv"][t] else None
        inv, cash, r, pnl, ir, fee, fb, fs = oracle.env_step(
            p, int(d["inv_before"][t]), float(d["cash_before"][t]), int(d["off_a"][t]),
            int(d["off_b"][t]), adv, d["mid"][t], d["ask"][t], d["bid"][t], d["buy_max"][t],
            d["sell_min"][t])
        assert (inv, fb, fs) == (d["inventory"][t], d["fill_buy"][t], d["fill_sell"][t]), t
        assert cash == d["cash"][t] and r == d["reward"][t] and pnl == d["pnl"][t], t
        assert ir == d["inv_reward"][t] and fee == d["fee_paid"][t], t


@pytest.mark.parametrize("name", ["g2_synthetic.npz", "g3_adversary.npz"])
def test_synthetic_episodes_match_reference(golden, oracle, name):
    d = golden(name)
    n_adv_active = 0
    n_diverged = []
    for ep in episodes_from_fixture(d):
        st = stats_dict(ep["stats"], ep["stats_nb"])
        s1n, s2n = oracle.normalize_signals(ep["s1"], ep["s2"], st)
        assert np.array_equal(s1n, ep["s1n"]) and np.array_equal(s2n, ep["s2n"])
        p = oracle.params(phi=ep["phi"], tick=ep["tick"], fee=ep["fee"])
        fit, trades, tr = oracle.evaluate(ep["mm"], ep["H"], ep["adv"], s1n, s2n, ep["mid"], ep["ask"],
                                          ep["bid"], ep["buy_max"], ep["sell_min"], p, trace=True)
        ref = ep["tr"]
        ours_act = np.stack([tr["off_a"], tr["off_b"]], 1)
        ref_act = np.stack([ref["off_a"], ref["off_b"]], 1)
        n = agree_until_justified_divergence(ours_act, ref_act, ep["raw"])
        if n < len(ref_act):
            # only the deliberately pathological large-weight genome may diverge
            assert np.abs(ep["raw"]).max() > 1e3, ep["e"]
            n_diverged.append(ep["e"])
        for k in ("off_a", "off_b", "adv_a", "adv_b", "inventory", "fill_buy", "fill_sell",
                  "cash", "reward", "pnl", "fee_paid"):
            assert np.array_equal(tr[k][:n], ref[k][:n]), (ep["e"], k)
        if n == len(ref_act):
            assert fit == ep["fitness"] and trades == ep["trades"], ep["e"]
        n_adv_active += int(np.any(ref["adv_a"] != 0) or np.any(ref["adv_b"] != 0))
    assert len(n_diverged) <= 1
    if name == "g3_adversary.npz":
        assert n_adv_active >= 4  # the adversary really perturbs quotes there


def test_idle_penalty_case_present(golden):
    d = golden("g2_synthetic.npz")
    # at least one episode trades and the fixture covers the fitness range
    assert d["trades"].max() > 0


def test_batch_equals_single(golden, oracle):
    d = golden("g2_synthetic.npz")
    eps = list(episodes_from_fixture(d))
    H32 = [e for e in eps if e["H"] == 32 and e["adv"] is None]
    mm = np.stack([e["mm"] for e in H32])
    ticks = [np.concatenate([e[k] for e in H32]) for k in ("s1n", "s2n", "mid", "ask", "bid", "buy_max", "sell_min")]
    lens = np.array([len(e["mid"]) for e in H32])
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]])
    plist = [oracle.params(phi=e["phi"], tick=e["tick"], fee=e["fee"]) for e in H32]
    fit, trd = oracle.evaluate_batch(mm, 32, None, ticks, np.arange(len(H32)), None, offs, lens,
                                     np.arange(len(H32)), plist, n_threads=2)
    single = [oracle.evaluate(e["mm"], 32, None, e["s1n"], e["s2n"], e["mid"], e["ask"], e["bid"],
                              e["buy_max"], e["sell_min"], pp) for e, pp in zip(H32, plist)]
    assert np.array_equal(fit, [f for f, _ in single])
    assert np.array_equal(trd, [t for _, t in single])
