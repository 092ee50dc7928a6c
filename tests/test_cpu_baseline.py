"""The CPU-baseline loop (oracle/ref_loop.py) reproduces the reference's own
fitness values (golden fixtures), so the baseline bench.py times is the
reference's computation with the reference's cost structure."""
import numpy as np

from conftest import episodes_from_fixture, stats_dict


def test_ref_loop_matches_reference_fixtures(golden):
    import ref_loop
    for name in ("g2_synthetic.npz", "g3_adversary.npz"):
        d = golden(name)
        for ep in list(episodes_from_fixture(d))[::3]:
            st = stats_dict(ep["stats"], ep["stats_nb"])
            b = (ep["s1"], ep["s2"], ep["mid"], ep["ask"], ep["bid"], ep["buy_max"], ep["sell_min"])
            f, t = ref_loop.episode(ep["mm"], ep["adv"], b, ep["phi"], ep["tick"], ep["fee"], st, ep["H"])
            assert f == ep["fitness"] and t == ep["trades"], (name, ep["e"])


def test_ref_loop_pool_matches_serial(golden):
    import ref_loop
    d = golden("g2_synthetic.npz")
    eps = [e for e in episodes_from_fixture(d) if e["H"] == 16 and e["adv"] is None][:4]
    st = stats_dict(eps[0]["stats"], eps[0]["stats_nb"])
    b = tuple(eps[0][k] for k in ("s1", "s2", "mid", "ask", "bid", "buy_max", "sell_min"))
    mm = np.stack([e["mm"] for e in eps])
    f1, t1, _, _ = ref_loop.population(mm, None, b, 0.001, 0.001, 0.0, st, 16, workers=1)
    f2, t2, _, w = ref_loop.population(mm, None, b, 0.001, 0.001, 0.0, st, 16, workers=2)
    assert f1 == f2 and t1 == t2 and w == 2
