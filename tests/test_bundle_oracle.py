"""The bundle-builder oracle (oracle/bundle_oracle.py) against the reference's
outputs on synthetic days (tests/golden/g6_bundle.npz)."""
import numpy as np
import pytest

import bundle_oracle as bo


def day_inputs(d, k):
    snap = {c[len(f"d{k}_snap_"):]: d[c] for c in d if c.startswith(f"d{k}_snap_")}
    tick = {c[len(f"d{k}_tick_"):]: d[c] for c in d if c.startswith(f"d{k}_tick_")}
    keep = (snap["trade_time"] >= 93000000) & (snap["askprice1"] > 0) & (snap["bidprice1"] > 0)
    snap = {c: v[keep] for c, v in snap.items()}  # agent_trainer.py:27 (inputs are already time-sorted)
    return snap, tick


def same(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return a.shape == b.shape and np.array_equal(a, b, equal_nan=True)


@pytest.fixture(scope="module")
def g6(golden):
    return golden("g6_bundle.npz")


def test_event_bars_match_reference(g6):
    for k in range(len(g6["dates"])):
        ev = bo.event_bars(*day_inputs(g6, k))
        for c in bo.EV_COLS:
            assert same(ev[c], g6[f"d{k}_ev_{c}"]), (k, c)


def test_sgu2_windows_match_reference(g6):
    for k in range(len(g6["dates"])):
        ev = {c: g6[f"d{k}_ev_{c}"] for c in bo.EV_COLS}
        X, y = bo.sgu2_windows(bo.bar_mids(ev))
        assert np.array_equal(X, g6[f"d{k}_sgu2_X"]) and np.array_equal(y, g6[f"d{k}_sgu2_y"]), k


def test_step_bundle_matches_load_signals_bundle(g6):
    parts = []
    for k in range(len(g6["dates"])):
        ev = {c: g6[f"d{k}_ev_{c}"] for c in bo.EV_COLS}
        X, _ = bo.sgu2_windows(bo.bar_mids(ev))
        s1 = g6[f"d{k}_sgu1_f0"].astype(np.float32)  # the stand-in m1 of the fixture
        s2 = X[:, -1, 0].astype(np.float32)          # the stand-in m2
        parts.append(bo.step_bundle(ev, s1, s2))
    for j, name in enumerate(("s1", "s2", "mid", "ask", "bid", "buy_max", "sell_min")):
        assert same(np.concatenate([p[j] for p in parts]), g6[f"bundle_{name}"]), name
