"""Measurement of the §8f rows (bundle builder, SGU2, backtest recorder) on
one MI355X: one JSON line per kernel with its throughput and roofline.

    python tools/bench_bundle.py [--days 240] [--reps 20]

Workload: a year of 510300.SH-shaped trading days (synthetic, seeded):
4800 three-second snapshots and 30k trades per day, 30% of the snapshots
repeating the previous quote (non-events).  Timing: the library's own HIP
events around every launch (sgmm_profile_*), averaged over --reps launches;
the rocprofv3 summary of the same command goes under profiles/.

Algorithmic bytes / flops per launch (DESIGN.md "Bundle builder"):
  event_bars   40 B per snapshot (time + 4 quote columns) + 28 B per trade
               (time, price, volume, side) read, 80 B per event row written
  bar_windows  32 B per event read (ask, bid, p_buy_max, p_sell_min),
               40 + 4 B per window written
  step_bundle  20 rows x 16 B (p_buy_max, p_sell_min) + 32 B read, 40 B
               written per step
  sgu2         per window and step 2*4H(H+1) + 6H FLOP (H = 10: 940), 40 B read
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
HBM_PEAK_GBPS = 8000.0
FP32_PEAK_TFLOPS = 157.3


def synthetic_days(n_days, n_snap=4800, n_tick=30000, seed=0):
    rng = np.random.default_rng(seed)
    days = []
    t_lo = 93000000
    for d in range(n_days):
        st = np.sort(rng.integers(t_lo, t_lo + 5_570_000, n_snap)).astype(np.int64)
        bid_k = 3490 + np.cumsum(rng.choice([-1, 0, 0, 1], n_snap))
        ask_k = bid_k + np.where(rng.random(n_snap) < 0.97, 1, 2)
        bv = rng.integers(1, 40, n_snap) * 100.0
        av = rng.integers(1, 40, n_snap) * 100.0
        keep = ~(rng.random(n_snap) < 0.3)
        keep[0] = True
        src = np.maximum.accumulate(np.where(keep, np.arange(n_snap), 0))  # repeat the last kept row
        snap = {"trade_time": st, "bidprice1": bid_k[src] / 1000.0, "askprice1": ask_k[src] / 1000.0,
                "bidvol1": bv[src], "askvol1": av[src]}
        tt = np.sort(rng.integers(t_lo - 50_000, t_lo + 5_600_000, n_tick)).astype(np.int64)
        tt[1::7] = tt[0:-1:7]
        tt = np.sort(tt)
        side = rng.choice([-1, 1], n_tick).astype(np.int32)
        price = np.round(3.49 + 0.001 * rng.integers(-20, 20, n_tick), 3)
        price[rng.random(n_tick) < 0.005] = np.nan
        tick = {"trade_time": tt, "Price": price, "Volume": rng.integers(1, 50, n_tick) * 100.0, "side": side}
        days.append((snap, tick))
    return days


def timed(fn, reps, kind):
    from sgmm_amd import _lib
    fn()
    torch.cuda.synchronize()
    _lib.profile_read()
    _lib.profile_enable(True)
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / reps
    _lib.profile_enable(False)
    prof = _lib.profile_read()
    ms, cnt = prof[kind]
    return ms / cnt * 1e-3, wall


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--days", type=int, default=240)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    import sgmm_pkg
    sgmm_pkg.load()
    from sgmm_amd.bundle import EventBarsGPU
    from sgmm_amd.gate_units import SGU2
    from sgmm_amd.rollout import EnvConfig, EpisodeBatch, RolloutEngine, TickStore, params_tensor
    from sgmm_amd.synthetic import bundle_510300, train_stats

    days = synthetic_days(args.days)
    S = sum(len(s["trade_time"]) for s, _ in days)
    K = sum(len(t["trade_time"]) for _, t in days)
    ev = EventBarsGPU(days)
    E = int(ev.n_events.sum())

    def build():
        from sgmm_amd import _lib
        import ctypes
        _lib.check(ev.L.sgmm_event_bars_build(ctypes.byref(ev.streams), ctypes.byref(ev.bars), _lib.ptr(ev._ws),
                                              ev._ws.numel(), _lib.stream_ptr()), "build")

    lines = []
    sec, wall = timed(build, args.reps, "event_bars")
    byt = 40 * S + 28 * K + 80 * E
    lines.append({"kernel": "k_event_bars", "workload": f"{args.days} days x 4800 snapshots x 30k trades",
                  "unit_rate": "days/s", "value": args.days / sec, "us_per_launch": sec * 1e6,
                  "roofline": {"bound": "hbm", "achieved": byt / sec / 1e9, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                               "frac": byt / sec / 1e9 / HBM_PEAK_GBPS, "algorithmic_bytes": byt}})
    ev.windows()
    W = int(ev.n_windows.sum())
    sec, _ = timed(ev.windows, args.reps, "bar_windows")
    byt = 32 * E + 44 * W
    lines.append({"kernel": "k_bar_windows", "unit_rate": "windows/s", "value": W / sec, "us_per_launch": sec * 1e6,
                  "roofline": {"bound": "hbm", "achieved": byt / sec / 1e9, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                               "frac": byt / sec / 1e9 / HBM_PEAK_GBPS, "algorithmic_bytes": byt}})
    total = (ev.n_events + 18) // 19
    ns = total
    ev.steps(ns)
    sec, _ = timed(lambda: ev.steps(ns), args.reps, "step_bundle")
    n_steps = int(np.maximum(ns - 1, 0).sum())
    byt = (20 * 16 + 32 + 40) * n_steps
    lines.append({"kernel": "k_step_bundle", "unit_rate": "steps/s", "value": n_steps / sec,
                  "us_per_launch": sec * 1e6,
                  "roofline": {"bound": "hbm", "achieved": byt / sec / 1e9, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                               "frac": byt / sec / 1e9 / HBM_PEAK_GBPS, "algorithmic_bytes": byt}})
    torch.manual_seed(0)
    m = SGU2(1, 10)
    nwin = 1 << 20
    X = (torch.randn(nwin, 10, device="cuda") * 3e-4).float()
    out = torch.empty(nwin, device="cuda")
    sec, _ = timed(lambda: m.predict_device(X, out=out), args.reps, "sgu2")
    flop = nwin * 10 * (2 * 40 * 11 + 60)
    lines.append({"kernel": "k_sgu2<10>", "workload": f"{nwin} windows x 10 steps", "unit_rate": "windows/s",
                  "value": nwin / sec, "us_per_launch": sec * 1e6,
                  "roofline": {"bound": "valu", "achieved": flop / sec / 1e12, "peak": FP32_PEAK_TFLOPS,
                               "unit": "TFLOP/s", "frac": flop / sec / 1e12 / FP32_PEAK_TFLOPS, "flop": flop}})
    # the recorder's trace launch: 64 backtests (checkpoints x phi sweep) of one 960-step test bundle
    b = bundle_510300(960, seed=4)
    ts = TickStore()
    ts.add(b, train_stats(b))
    ts.to("cuda")
    nb = 64
    params = params_tensor([EnvConfig(phi=p, tick_size=0.001) for p in np.geomspace(1e-4, 1e-2, nb)], "cuda")
    eps = EpisodeBatch(np.arange(nb), np.zeros(nb), np.full(nb, 960), np.arange(nb)).to("cuda")
    mm = (torch.randn(nb, 1250, device="cuda") * 0.2).float()
    eng = RolloutEngine("cuda")
    sec, _ = timed(lambda: eng.trace(ts, eps, params, mm, 32), args.reps, "rollout_direct")
    lines.append({"kernel": "k_rollout_direct<32>", "workload": "64 backtests x 960 steps (recorder trace)",
                  "unit_rate": "env-steps/s", "value": nb * 960 / sec, "us_per_launch": sec * 1e6,
                  "roofline": {"bound": "latency", "note": "one wave per backtest, the 960 steps are a serial "
                               "chain (inventory feedback); 64 waves occupy 64 of 1024 SIMDs",
                               "us_per_step": sec * 1e6 / 960}})
    for ln in lines:
        print(json.dumps(ln))


if __name__ == "__main__":
    main()
