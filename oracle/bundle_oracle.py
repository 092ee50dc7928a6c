"""TEST INFRASTRUCTURE ONLY -- CPU restatement of the reference's bundle
builder.  Used by tests/ as the checker of the HIP
bundle kernels; the product path never imports it.

Restated (numpy, plain loops where order matters), with the reference lines:
  event_bars   loaders/HFTLoader.py:26-63  L1-change event mask
               (diff != 0 on bid/ask price/volume, first row always), per
               trade_time tick aggregation (max buy price, min sell price,
               volume sums, price count, sum price*volume -- pandas' Kahan
               compensated group sum, NaN skipped, in row order),
               merge_asof(direction='backward') onto the events
  bar_mids     loaders/HFTLoader.py:141-156  per 19-event group:
               0.5*(max p_buy_max + min p_sell_min) with the mean-price
               fallbacks; pandas Series.mean == numpy pairwise sum / count
  sgu2_windows loaders/HFTLoader.py:158-169  ffill, float32, floor 1e-5,
               (m - m_lag) / (m_lag + 1e-9), 10-step windows, nan_to_num
  step_bundle  pipeline/agent_trainer.py:45-78  alignment to the signals,
               inclusive .loc window max/min, ask/bid now, mid at the next step

Pinned by tests/golden/g6_bundle.npz (the reference run on synthetic days,
tests/golden/gen_golden_bundle.py).
"""
from __future__ import annotations

import numpy as np

EV_COLS = ("trade_time", "askprice1", "bidprice1", "p_buy_max", "p_sell_min", "v_buy_sum",
           "v_sell_sum", "vol_sum", "trade_count", "vwap_num")


def pairwise_sum(a: np.ndarray) -> float:
    """numpy's float64 add.reduce order (pairwise blocks of 8 accumulators),
    for n <= 128 -- what pandas' Series.mean/sum evaluate."""
    a = np.asarray(a, np.float64)
    n = len(a)
    if n < 8:
        s = 0.0
        for v in a:
            s = s + v
        return s
    r = [a[j] for j in range(8)]
    i = 8
    while i + 8 <= n:
        for j in range(8):
            r[j] = r[j] + a[i + j]
        i += 8
    s = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]))
    while i < n:
        s = s + a[i]
        i += 1
    return s


def kahan_sum(a) -> float:
    """pandas' groupby sum for float64 (pandas >= 1.3, groupby.pyx group_sum):
    NaN skipped, Kahan-compensated in row order, 0.0 when nothing is summed."""
    s = c = 0.0
    for v in np.asarray(a, np.float64):
        if v != v:
            continue
        y = v - c
        t = s + y
        c = (t - s) - y
        if c != c:  # +-inf input (pandas GH#53606)
            c = 0.0
        s = t
    return s


def nanmax(a):
    a = np.asarray(a, np.float64)
    a = a[~np.isnan(a)]
    return np.float64(np.nan) if len(a) == 0 else a.max()


def nanmin(a):
    a = np.asarray(a, np.float64)
    a = a[~np.isnan(a)]
    return np.float64(np.nan) if len(a) == 0 else a.min()


def event_bars(snap: dict, tick: dict) -> dict:
    """HFTMarketBase (HFTLoader.py:26-63) on trade_time-sorted columns."""
    t = np.asarray(snap["trade_time"], np.int64)
    cols = [np.asarray(snap[c], np.float64) for c in ("bidprice1", "askprice1", "bidvol1", "askvol1")]
    n = len(t)
    mask = np.zeros(n, bool)
    for i in range(n):
        mask[i] = i == 0 or any(not (c[i] - c[i - 1] == 0) for c in cols)
    ev = np.nonzero(mask)[0]
    tt = np.asarray(tick["trade_time"], np.int64)
    price = np.asarray(tick["Price"], np.float64)
    vol = np.asarray(tick["Volume"], np.float64)
    side = np.asarray(tick["side"])
    starts = [i for i in range(len(tt)) if i == 0 or tt[i] != tt[i - 1]]
    g_time, g_stats = [], []
    for k, s in enumerate(starts):
        e = starts[k + 1] if k + 1 < len(starts) else len(tt)
        pb = price[s:e][side[s:e] == 1]
        ps = price[s:e][side[s:e] == -1]
        vb = kahan_sum([vol[i] if side[i] == 1 else 0.0 for i in range(s, e)])
        vs = kahan_sum([vol[i] if side[i] == -1 else 0.0 for i in range(s, e)])
        vv = kahan_sum(vol[s:e])
        vw = kahan_sum(price[s:e] * vol[s:e])
        g_time.append(tt[s])
        g_stats.append((nanmax(pb), nanmin(ps), vb, vs, vv, float(np.sum(~np.isnan(price[s:e]))), vw))
    g_time = np.array(g_time, np.int64)
    out = {c: np.empty(len(ev)) for c in EV_COLS[3:]}
    out["trade_time"] = t[ev]
    out["askprice1"] = cols[1][ev]
    out["bidprice1"] = cols[0][ev]
    for j, r in enumerate(ev):
        k = np.searchsorted(g_time, t[r], side="right") - 1
        vals = g_stats[k] if k >= 0 else (np.nan,) * 7
        for c, v in zip(EV_COLS[3:], vals):
            out[c][j] = v
    return out


def bar_mids(ev: dict, event_step: int = 19) -> np.ndarray:
    """SGU2DataPro's per-group mid estimate m (HFTLoader.py:141-156)."""
    n = len(ev["trade_time"])
    m = []
    for i in range(0, n - event_step, event_step):
        sl = slice(i, i + event_step)
        bmax, smin = nanmax(ev["p_buy_max"][sl]), nanmin(ev["p_sell_min"][sl])
        a_mean = pairwise_sum(ev["askprice1"][sl]) / event_step
        b_mean = pairwise_sum(ev["bidprice1"][sl]) / event_step
        if not np.isnan(bmax) and not np.isnan(smin):
            m.append(0.5 * (bmax + smin))
        elif np.isnan(bmax) and not np.isnan(smin):
            m.append(0.5 * (a_mean + smin))
        elif not np.isnan(bmax) and np.isnan(smin):
            m.append(0.5 * (bmax + b_mean))
        else:
            m.append(0.5 * (a_mean + b_mean))
    return np.array(m, np.float64)


def sgu2_windows(m: np.ndarray, time_steps: int = 10):
    """HFTLoader.py:158-169: returns the (X, y) windows (float32)."""
    if len(m) <= time_steps + 1:
        return np.zeros((0,), np.float32), np.zeros((0,), np.float32)
    m = m.copy()
    for i in range(1, len(m)):  # ffill
        if np.isnan(m[i]):
            m[i] = m[i - 1]
    mf = m.astype(np.float32)
    mf[mf < np.float32(1e-5)] = np.float32(1e-5)
    lag = np.full_like(mf, np.nan)
    lag[1:] = mf[:-1]
    ret = ((mf - lag) / (lag + np.float32(1e-9))).astype(np.float32)[1:]
    X = np.stack([ret[t - time_steps:t] for t in range(time_steps, len(ret))])[:, :, None]
    y = ret[time_steps:]
    return np.nan_to_num(X), np.nan_to_num(y)


def step_bundle(ev: dict, s1_pred: np.ndarray, s2_pred: np.ndarray, event_step: int = 19):
    """agent_trainer.py:45-78 for one day: (s1, s2, mid, ask, bid, buy_max, sell_min)."""
    n = len(ev["trade_time"])
    min_len = min(len(s1_pred), len(s2_pred))
    pos = np.arange(0, n, event_step)[-min_len:]
    bmax = [nanmax(ev["p_buy_max"][pos[i]:pos[i + 1] + 1]) for i in range(len(pos) - 1)]
    smin = [nanmin(ev["p_sell_min"][pos[i]:pos[i + 1] + 1]) for i in range(len(pos) - 1)]
    ask, bid = ev["askprice1"][pos], ev["bidprice1"][pos]
    mid = (ask[1:] + bid[1:]) / 2
    return (np.asarray(s1_pred[-min_len:][:-1]), np.asarray(s2_pred[-min_len:][:-1]), mid, ask[:-1], bid[:-1],
            np.array(bmax), np.array(smin))
