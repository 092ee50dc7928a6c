"""Synthetic 510300.SH-shaped tick bundles for benchmarks and tests.

Real LOB data is not distributed with the reference (data/ is gitignored), so
benchmarks run on bundles with the observed shape of the 510300 OOS episode
(output/510300/*/backtest_0.0001.parquet): a bid random walk on the 0.001 tick
grid around 3.49, a one-tick spread 97.4% of the time, FPT step extremes within
-1..+2 ticks of the touch (a zero-offset quote fills ~95% of steps per side),
and the two gate-unit signals as N(2.09, 0.325) / N(0.027, 0.516) float32.
Prices are k / (1/tick) on the decimal grid, as the reference's int/10000
conversion (loaders/get_l2_data.py:37-39) produces.
"""
from __future__ import annotations

import numpy as np


def bundle_510300(T: int, seed: int = 0, tick: float = 0.001, start_ticks: int = 3490,
                  nan_frac: float = 0.0):
    """(s1, s2, mid_next, best_ask, best_bid, buy_max, sell_min) of length T."""
    rng = np.random.default_rng(seed)
    per = int(round(1.0 / tick))
    bid_k = start_ticks + np.cumsum(rng.choice([-1, 0, 1], size=T + 1, p=[0.3, 0.4, 0.3]))
    ask_k = bid_k + np.where(rng.random(T + 1) < 0.974, 1, 2)
    ask, bid = ask_k / per, bid_k / per
    mid_next = (ask[1:] + bid[1:]) / 2
    ext = [-1, 0, 1, 2]
    pr = [0.05, 0.55, 0.30, 0.10]
    buy_max = (ask_k[:T] + rng.choice(ext, size=T, p=pr)) / per
    sell_min = (bid_k[:T] - rng.choice(ext, size=T, p=pr)) / per
    if nan_frac > 0:
        buy_max[rng.random(T) < nan_frac] = np.nan
        sell_min[rng.random(T) < nan_frac] = np.nan
    s1 = rng.normal(2.09, 0.325, T).astype(np.float32)
    s2 = rng.normal(0.027, 0.516, T).astype(np.float32)
    return (s1, s2, mid_next.astype(np.float64), ask[:T].astype(np.float64),
            bid[:T].astype(np.float64), buy_max.astype(np.float64), sell_min.astype(np.float64))


def bundle_688981(T: int, seed: int = 0):
    """688981.SH-shaped bundle: tick 0.01 around 45.00 (no data in the reference
    repo; the level is an assumption, the tick is the STAR-market tick)."""
    return bundle_510300(T, seed=seed, tick=0.01, start_ticks=4500)


def train_stats(bundle):
    """train_stats as agent_trainer.py:126-129 computes them."""
    s1, s2 = bundle[0], bundle[1]
    return {"s1_m": np.mean(s1), "s1_s": np.std(s1) + 1e-9,
            "s2_m": np.mean(s2), "s2_s": np.std(s2) + 1e-9}


def population(P: int, hidden: int, sigma: float = 0.05, seed: int = 0):
    """P genomes around an orthogonally initialised master (torch CPU RNG)."""
    import torch
    from .model import TradingPolicy
    g = torch.Generator().manual_seed(seed)
    state = torch.random.get_rng_state()
    torch.manual_seed(seed)
    try:
        master = TradingPolicy(hidden_dim=hidden).get_weights()
    finally:
        torch.random.set_rng_state(state)
    noise = torch.randn((P, master.numel()), generator=g) * sigma
    return master + noise
