"""GPU tests of the bundle builder: libsgmm.so's
event-bar / SGU2-window / step-bundle kernels against the reference's own
outputs (tests/golden/g6_bundle.npz) and against oracle/bundle_oracle.py on
seeded synthetic days with the edge cases the reference's data can hold.
Bit-exact throughout (float64 columns, float32 windows)."""
import numpy as np
import pandas as pd
import pytest

from conftest import has_gpu

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not has_gpu(), reason="needs a HIP device")]

NAMES = ("s1", "s2", "mid", "ask", "bid", "buy_max", "sell_min")


def same(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return a.shape == b.shape and np.array_equal(a.astype(np.float64), b.astype(np.float64), equal_nan=True)


@pytest.fixture(scope="module")
def g6(golden):
    return golden("g6_bundle.npz")


def golden_days(g6):
    from sgmm_amd.bundle import _filter_sort
    days = []
    for k in range(len(g6["dates"])):
        snap = pd.DataFrame({c[len(f"d{k}_snap_"):]: g6[c] for c in g6 if c.startswith(f"d{k}_snap_")})
        tick = pd.DataFrame({c[len(f"d{k}_tick_"):]: g6[c] for c in g6 if c.startswith(f"d{k}_tick_")})
        days.append(_filter_sort(snap, tick))
    return days


def test_event_bars_match_reference(sgmm, g6):
    from sgmm_amd.bundle import EV_COLS, event_bars
    ev = event_bars(golden_days(g6))
    for k in range(len(g6["dates"])):
        day = ev.day(k)
        for c in EV_COLS:
            assert same(day[c], g6[f"d{k}_ev_{c}"]), (k, c)


def test_sgu2_windows_match_reference(sgmm, g6):
    from sgmm_amd.bundle import event_bars
    wins = event_bars(golden_days(g6)).windows()
    for k, (X, y) in enumerate(wins):
        assert str(X.dtype) == "torch.float32"
        assert np.array_equal(X.cpu().numpy(), g6[f"d{k}_sgu2_X"]), k
        assert np.array_equal(y.cpu().numpy(), g6[f"d{k}_sgu2_y"]), k


class M1:
    def predict(self, X):
        return np.asarray(X.iloc[:, 0].values, dtype=np.float32)


class M2:
    def predict(self, X):
        return np.asarray(X[:, -1, 0], dtype=np.float32).reshape(-1, 1)


class Identity:
    def transform(self, X):
        return X


def test_load_signals_bundle_matches_reference(sgmm, g6, tmp_path):
    """The drop-in load_signals_bundle on parquet files (the reference's own
    layout data/{symbol}/{snap,tick}/{date}.parquet) with the fixture's
    stand-in models, against the reference's 7-tuple."""
    from sgmm_amd.bundle import load_signals_bundle
    dates = [str(d) for d in g6["dates"]]
    for k, d in enumerate(dates):
        for kind in ("snap", "tick"):
            p = tmp_path / "data" / "SYN" / kind
            p.mkdir(parents=True, exist_ok=True)
            pd.DataFrame({c[len(f"d{k}_{kind}_"):]: g6[c] for c in g6 if c.startswith(f"d{k}_{kind}_")}) \
                .to_parquet(p / f"{d}.parquet")
    f0 = iter([g6[f"d{k}_sgu1_f0"] for k in range(len(dates))])

    def sgu1_features(bars):  # the fixture pins SGU1's first feature column (days in order)
        v = next(f0)
        return pd.DataFrame({"f0": v, "label": np.zeros(len(v))})

    out = load_signals_bundle("SYN", dates, M1(), M2(), Identity(), sgu1_features=sgu1_features,
                              data_root=str(tmp_path))
    for name, a in zip(NAMES, out):
        assert same(a, g6[f"bundle_{name}"]), name


def synthetic(seed, n_snap, n_tick, t_lo=93000000):
    rng = np.random.default_rng(seed)
    st = np.sort(rng.integers(t_lo, t_lo + 6_000_000, n_snap)).astype(np.int64)
    bid = 3.4 + 0.001 * np.cumsum(rng.choice([-1, 0, 0, 1], n_snap))
    ask = bid + 0.001 * rng.choice([1, 1, 1, 2], n_snap)
    bv = rng.integers(1, 5, n_snap) * 100.0
    av = rng.integers(1, 5, n_snap) * 100.0
    rep = rng.random(n_snap) < 0.4
    for i in range(1, n_snap):
        if rep[i]:
            bid[i], ask[i], bv[i], av[i] = bid[i - 1], ask[i - 1], bv[i - 1], av[i - 1]
    tt = np.sort(rng.integers(t_lo - 100_000, t_lo + 6_100_000, n_tick)).astype(np.int64)
    tt[1::5] = tt[0:-1:5]
    tt = np.sort(tt)
    side = rng.choice([-1, 1], n_tick).astype(np.int32)
    price = np.round(3.4 + 0.01 * rng.standard_normal(n_tick), 3)
    price[rng.random(n_tick) < 0.01] = np.nan
    vol = rng.integers(1, 30, n_tick) * 100.0
    snap = {"trade_time": st, "bidprice1": bid, "askprice1": ask, "bidvol1": bv, "askvol1": av}
    tick = {"trade_time": tt, "Price": price, "Volume": vol, "side": side}
    return snap, tick


def edge_days():
    days = [synthetic(1, 5000, 20000), synthetic(2, 3000, 0), synthetic(3, 1, 7), synthetic(4, 400, 3),
            synthetic(5, 2100, 9000, t_lo=93000000)]
    s, t = synthetic(6, 600, 2000)
    for c in ("bidprice1", "askprice1", "bidvol1", "askvol1"):
        s[c][:] = s[c][0]  # one event all day
    days.append((s, t))
    s, t = synthetic(7, 700, 1500)
    t["trade_time"] = t["trade_time"] + 10_000_000  # every trade after the last snapshot
    days.append((s, t))
    s, t = synthetic(8, 19 * 12 + 1, 500)  # exactly 12 bars boundary
    for c in ("bidprice1",):
        s[c] = 3.0 + 0.001 * np.arange(len(s[c]))  # every row an event
    days.append((s, t))
    return days


@pytest.fixture(scope="module")
def edge():
    import bundle_oracle as bo
    days = edge_days()
    return days, [bo.event_bars(s, t) for s, t in days]


def test_event_bars_match_oracle_edge_cases(sgmm, edge):
    from sgmm_amd.bundle import EV_COLS, event_bars
    days, want = edge
    ev = event_bars(days)
    for k, w in enumerate(want):
        got = ev.day(k)
        assert len(got["trade_time"]) == len(w["trade_time"]), k
        for c in EV_COLS:
            assert same(got[c], w[c]), (k, c)


def test_windows_and_steps_match_oracle_edge_cases(sgmm, edge):
    import bundle_oracle as bo
    from sgmm_amd.bundle import event_bars
    days, want = edge
    ev = event_bars(days)
    wins = ev.windows()
    n_samples, parts = [], []
    for k, w in enumerate(want):
        X, y = bo.sgu2_windows(bo.bar_mids(w))
        gx, gy = wins[k]
        assert gx.shape[0] == (X.shape[0] if X.ndim == 3 else 0), k
        if X.ndim == 3:
            assert np.array_equal(gx.cpu().numpy(), X) and np.array_equal(gy.cpu().numpy(), y), k
        total = (len(w["trade_time"]) + 18) // 19
        ns = [0, total, max(total - 3, 0), total + 5][k % 4]
        n_samples.append(ns)
        if ns > 0:  # n_samples 0 = a skipped day (agent_trainer.py:33-41)
            sig = np.zeros(ns, np.float32)
            p = bo.step_bundle(w, sig, sig)
            parts.append(p[2:])
    (mid, ask, bid, bmax, smin), n_steps = ev.steps(n_samples)
    assert int(n_steps.sum()) == mid.shape[0]
    for j, g in enumerate((mid, ask, bid, bmax, smin)):
        want_j = np.concatenate([p[j] for p in parts]) if parts else np.zeros(0)
        assert same(g.cpu().numpy(), want_j), j


def test_bundle_many_days_one_launch(sgmm, g6):
    """All days of a request go through one launch per kernel: 64 copies of
    the golden days give 64 copies of the reference's event bars."""
    from sgmm_amd.bundle import EV_COLS, event_bars
    days = golden_days(g6)
    ev = event_bars(days * 16)
    for r in range(16):
        for k in range(len(days)):
            day = ev.day(r * len(days) + k)
            for c in EV_COLS:
                assert same(day[c], g6[f"d{k}_ev_{c}"]), (r, k, c)
