"""Reference-equivalent CPU rollout loop -- TEST / BASELINE INFRASTRUCTURE ONLY.

A restatement of the reference's own CPU hot loop with its cost structure
intact, used by bench.py's ``cpu_baseline`` leg (kind "port") on the GPU box,
where the reference source is not available:

  * evaluate_individual (Env/drl_engine.py:9-67): per tick, build the state as
    a [1,3] float32 torch tensor, run a batch-1 torch MLP forward, round the
    actions with numpy, step the FPT env with numpy scalars, accumulate the
    float64 reward;
  * the population is mapped over a fork Pool with one torch thread per worker
    (drl_engine.py:91,115; torch.set_num_threads(1) avoids the fork deadlock
    SURVEY.md 5 records).

Validated against the reference-generated golden fixtures by
tests/test_cpu_baseline.py (identical fitness and trades).
"""
from __future__ import annotations

import os
import time

import numpy as np
import torch
import torch.nn as nn


def _mlp(weights: torch.Tensor, hidden: int) -> nn.Module:
    net = nn.Sequential(nn.Linear(3, hidden), nn.ReLU(), nn.Linear(hidden, hidden), nn.ReLU(),
                        nn.Linear(hidden, 2))
    i = 0
    with torch.no_grad():
        for p in net.parameters():
            n = p.numel()
            p.copy_(weights[i:i + n].view_as(p))
            i += n
    return net.eval()


def _adv(weights: torch.Tensor) -> nn.Module:
    net = nn.Sequential(nn.Linear(3, 12), nn.ReLU(), nn.Linear(12, 2), nn.Tanh())
    i = 0
    with torch.no_grad():
        for p in net.parameters():
            n = p.numel()
            p.copy_(weights[i:i + n].view_as(p))
            i += n
    return net.eval()


def episode(mm_weights, adv_weights, bundle, phi, tick, fee, stats, hidden=32):
    """One evaluate_individual episode, step by step as the reference runs it."""
    s1, s2, mid_next, ask, bid, bmax, smin = bundle
    pol = _mlp(torch.as_tensor(mm_weights, dtype=torch.float32), hidden)
    adv = _adv(torch.as_tensor(adv_weights, dtype=torch.float32)) if adv_weights is not None else None
    inv, cash, total, trades = 0, 0.0, 0, 0
    fb_flag = fs_flag = 0.0
    with torch.no_grad():
        for t in range(len(mid_next)):
            x = torch.tensor([[(s1[t] - stats["s1_m"]) / stats["s1_s"],
                               (s2[t] - stats["s2_m"]) / stats["s2_s"], inv / 2.0]], dtype=torch.float32)
            act = np.round(pol(x).squeeze().numpy() * 5.0).astype(int)
            oa, ob = act[0], act[1]
            if adv is not None:
                xa = torch.tensor([[inv / 2.0, fs_flag, fb_flag]], dtype=torch.float32)
                d = np.round(np.round(adv(xa).squeeze().numpy() * 1.0).astype(int)).astype(int)
                oa, ob = oa + d[0], ob + d[1]
            qa = ask[t] + oa * tick
            qb = bid[t] - ob * tick
            buy = 1 if (inv < 2 and qb >= smin[t]) else 0
            sell = 1 if (inv > -2 and qa <= bmax[t]) else 0
            pnl = 0.0
            if buy:
                inv += 1
                f = qb * fee
                cash -= (qb + f)
                pnl += (mid_next[t] - qb) - f
            if sell:
                inv -= 1
                f = qa * fee
                cash += (qa - f)
                pnl += (qa - mid_next[t]) - f
            total += pnl - phi * abs(inv)
            fb_flag, fs_flag = float(buy), float(sell)
            trades += 1 if (buy or sell) else 0
    if trades == 0:
        total -= 50.0
    return total, trades


_POOL_ARGS = None


def _worker_init():
    torch.set_num_threads(1)


def _run_one(i):
    mm, adv, bundle, phi, tick, fee, stats, hidden = _POOL_ARGS
    ph = phi[i] if np.ndim(phi) else phi  # per-episode phi (a lambda sweep) or one for all
    return episode(mm[i], None if adv is None else adv[i], bundle, ph, tick, fee, stats, hidden)


def _noop(i):
    return i


class RefPool:
    """A fork Pool of reference-loop workers (drl_engine.py:91), created and
    warmed up OUTSIDE the timed region; ``map()`` times only the episodes.

    ``phi`` may be one value or one per episode."""

    def __init__(self, mm, adv, bundle, phi, tick, fee, stats, hidden=32, workers=1):
        import multiprocessing as mp
        global _POOL_ARGS
        self.workers = int(workers)
        _POOL_ARGS = (mm, adv, bundle, phi, tick, fee, stats, hidden)
        torch.set_num_threads(1)
        self.n = len(mm)
        self.pool = None
        if self.workers > 1:
            self.pool = mp.get_context("fork").Pool(processes=self.workers, initializer=_worker_init)
            self.pool.map(_noop, range(4 * self.workers), chunksize=1)  # every worker forked and running

    def map(self):
        """(fitness list, trades list, wall seconds of the episodes only)."""
        t0 = time.perf_counter()
        if self.pool is None:
            res = [_run_one(i) for i in range(self.n)]
        else:
            res = self.pool.map(_run_one, range(self.n), chunksize=1)
        dt = time.perf_counter() - t0
        return [r[0] for r in res], [r[1] for r in res], dt

    def close(self):
        global _POOL_ARGS
        if self.pool is not None:
            self.pool.close()
            self.pool.join()
        _POOL_ARGS = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def population(mm, adv, bundle, phi, tick, fee, stats, hidden=32, workers=None):
    """Map episode() over a population with a fork Pool (drl_engine.py:91,115).

    Returns (fitness list, trades list, wall seconds of the map, workers used);
    pool start-up is not timed."""
    workers = int(workers or min(16, os.cpu_count() or 1))
    with RefPool(mm, adv, bundle, phi, tick, fee, stats, hidden, workers) as rp:
        f, t, dt = rp.map()
    return f, t, dt, workers
