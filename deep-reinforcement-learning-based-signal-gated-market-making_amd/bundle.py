"""Signal-bundle builder on the GPU.

The data path in front of the rollout: raw snapshot / trade streams of many
trading days -> event bars (loaders/HFTLoader.py:26-63) -> SGU2 input windows
(HFTLoader.py:139-169) -> the per-step bundle of load_signals_bundle
(pipeline/agent_trainer.py:15-78).  Every day is one workgroup of
libsgmm.so's bundle kernels; all days of a request go in one launch each.

``load_signals_bundle`` keeps the reference's signature and result (the
7-tuple s1, s2, mid_next, ask, bid, buy_max, sell_min).  Host work is limited
to what the reference does with pandas before its loops: reading the
parquet files, the 09:30 filter and the trade_time sort (DataFrame
.sort_values, so tie order matches).  The signal models stay the caller's:
m2 receives the windows (scaled by ``scaler``); SGU1's feature table
(HFTLoader.py:66-135, an xgboost model -- not part of this path) comes from
the ``sgu1_features`` callable.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

from . import _lib
from ._lib import DayStreams, EventBars, check, ptr, stream_ptr

EVENT_STEP, TIME_STEPS = 19, 10
EV_COLS = ("trade_time", "askprice1", "bidprice1", "p_buy_max", "p_sell_min", "v_buy_sum",
           "v_sell_sum", "vol_sum", "trade_count", "vwap_num")


def _filter_sort(snap, tick):
    """agent_trainer.py:27 (09:30 filter) + HFTLoader.py:29-30 (sorts)."""
    snap = snap[(snap["trade_time"] >= 93000000) & (snap["askprice1"] > 0) & (snap["bidprice1"] > 0)]
    return (snap.sort_values("trade_time").reset_index(drop=True),
            tick.sort_values("trade_time").reset_index(drop=True))


class EventBarsGPU:
    """Event bars of n days, resident on the device (rows of day d start at
    snap_off[d]; n_events[d] of them are valid).  ``days`` holds (snap, tick)
    per day -- DataFrames or dicts of columns, trade_time-sorted."""

    def __init__(self, days, device="cuda"):
        _lib.require_gpu()
        self.L = _lib.load()
        dev = self.device = torch.device(device)
        self.n_days = len(days)
        snaps = [s for s, _ in days]
        ticks = [t for _, t in days]
        self.snap_off = np.concatenate([[0], np.cumsum([len(s["trade_time"]) for s in snaps])]).astype(np.int64)
        self.tick_off = np.concatenate([[0], np.cumsum([len(t["trade_time"]) for t in ticks])]).astype(np.int64)
        n_s, n_t = int(self.snap_off[-1]), int(self.tick_off[-1])

        def col(frames, c, dt):
            a = np.concatenate([np.asarray(f[c], dt) for f in frames]) if frames else np.zeros(0, dt)
            return torch.from_numpy(np.ascontiguousarray(a)).to(dev)

        self._in = {
            "snap_off": torch.from_numpy(self.snap_off).to(dev), "tick_off": torch.from_numpy(self.tick_off).to(dev),
            "snap_time": col(snaps, "trade_time", np.int64), "bid": col(snaps, "bidprice1", np.float64),
            "ask": col(snaps, "askprice1", np.float64), "bidvol": col(snaps, "bidvol1", np.float64),
            "askvol": col(snaps, "askvol1", np.float64), "tick_time": col(ticks, "trade_time", np.int64),
            "price": col(ticks, "Price", np.float64), "volume": col(ticks, "Volume", np.float64),
            "side": col(ticks, "side", np.int32),
        }
        f64 = dict(dtype=torch.float64, device=dev)
        self.cols = {"trade_time": torch.empty(max(n_s, 1), dtype=torch.int64, device=dev)}
        for c in EV_COLS[1:]:
            self.cols[c] = torch.empty(max(n_s, 1), **f64)
        self.n_events_dev = torch.zeros(max(self.n_days, 1), dtype=torch.int32, device=dev)
        i = self._in
        self.streams = DayStreams(self.n_days, 0, n_t, *[ptr(i[k]) for k in (
            "snap_off", "snap_time", "bid", "ask", "bidvol", "askvol", "tick_off", "tick_time", "price",
            "volume", "side")])
        c = self.cols
        self.bars = EventBars(ptr(self.n_events_dev), *[ptr(c[k]) for k in (
            "trade_time", "askprice1", "bidprice1", "p_buy_max", "p_sell_min", "v_buy_sum", "v_sell_sum",
            "vol_sum", "trade_count", "vwap_num")])
        ws = torch.empty(int(self.L.sgmm_event_bars_workspace_size(n_t)), dtype=torch.uint8, device=dev)
        check(self.L.sgmm_event_bars_build(ctypes.byref(self.streams), ctypes.byref(self.bars), ptr(ws),
                                           ws.numel(), stream_ptr()), "sgmm_event_bars_build")
        self._ws = ws
        self.n_events = self.n_events_dev[:self.n_days].cpu().numpy()

    def day(self, d: int) -> dict:
        """Event bars of day d as host arrays (HFTMarketBase.event_df columns)."""
        a, n = int(self.snap_off[d]), int(self.n_events[d])
        return {c: v[a:a + n].cpu().numpy() for c, v in self.cols.items()}

    def windows(self):
        """SGU2DataPro.gen_dataset(19, 10) of every day: list of (X [n,10,1], y [n]) on device."""
        cap = (np.diff(self.snap_off) // EVENT_STEP + 1).astype(np.int64)
        win_off = np.concatenate([[0], np.cumsum(cap)]).astype(np.int64)
        dev = self.device
        X = torch.zeros((max(int(win_off[-1]), 1), TIME_STEPS), dtype=torch.float32, device=dev)
        y = torch.zeros(max(int(win_off[-1]), 1), dtype=torch.float32, device=dev)
        nw = torch.zeros(max(self.n_days, 1), dtype=torch.int32, device=dev)
        bars_max = int((self.n_events.max() if self.n_days else 0) // EVENT_STEP + 1)
        win_off_d = torch.from_numpy(win_off).to(dev)  # held until the launch is enqueued
        check(self.L.sgmm_bar_windows(ctypes.byref(self.bars), self.n_days, ptr(self._in["snap_off"]),
                                      ptr(win_off_d), ptr(X), ptr(y), ptr(nw),
                                      bars_max, stream_ptr()), "sgmm_bar_windows")
        nw = nw[:self.n_days].cpu().numpy()
        if (nw < 0).any():
            raise _lib.SgmmError(f"more than 4096 bars on day(s) {np.nonzero(nw < 0)[0].tolist()}")
        self.X_all, self.win_off, self.n_windows = X, win_off, nw
        return [(X[win_off[d]:win_off[d] + nw[d]].unsqueeze(-1), y[win_off[d]:win_off[d] + nw[d]])
                for d in range(self.n_days)]

    def steps(self, n_samples) -> tuple:
        """The step loop of load_signals_bundle for every day with its number of
        aligned samples (min(len(s1), len(s2)), clipped to the sampled events):
        concatenated (mid_next, ask, bid, buy_max, sell_min) as device tensors."""
        total = (self.n_events + EVENT_STEP - 1) // EVENT_STEP
        ns = np.minimum(np.asarray(n_samples, np.int64), total).astype(np.int32)
        n_steps = np.maximum(ns - 1, 0)
        step_off = np.concatenate([[0], np.cumsum(n_steps)]).astype(np.int64)
        dev = self.device
        outs = [torch.empty(max(int(step_off[-1]), 1), dtype=torch.float64, device=dev) for _ in range(5)]
        # named so that neither block returns to the allocator before the launch
        ns_d, step_off_d = torch.from_numpy(ns).to(dev), torch.from_numpy(step_off).to(dev)
        check(self.L.sgmm_step_bundle(ctypes.byref(self.bars), self.n_days, ptr(self._in["snap_off"]),
                                      ptr(ns_d), ptr(step_off_d),
                                      int(n_steps.max()) if self.n_days else 0, *[ptr(o) for o in outs],
                                      stream_ptr()), "sgmm_step_bundle")
        return tuple(o[:int(step_off[-1])] for o in outs), n_steps


def event_bars(days, device="cuda") -> EventBarsGPU:
    """HFTMarketBase for a list of (snap, tick) DataFrames (already filtered
    and sorted, see load_signals_bundle)."""
    return EventBarsGPU(days, device)


def _fused_sgu2(m2, scaler) -> bool:
    """m2 is this package's SGU2 and the scaler a float32 StandardScaler3D fit
    (what utils/scaler.py yields for the float32 windows): the transform then
    is the kernel's float32 (x - mean) / std."""
    from .gate_units import SGU2
    mean, std = getattr(scaler, "mean", None), getattr(scaler, "std", None)
    return (isinstance(m2, SGU2) and type(scaler).__name__ == "StandardScaler3D"
            and isinstance(mean, np.ndarray) and isinstance(std, np.ndarray)
            and mean.dtype == np.float32 and std.dtype == np.float32 and mean.size == 1 and std.size == 1)


def load_signals_bundle(symbol, date_list, m1, m2, scaler, *, sgu1_features=None, data_root=".",
                        device="cuda"):
    """pipeline/agent_trainer.py:15-78 with the event bars, the SGU2 windows
    and the step loop on the GPU.  ``sgu1_features(event_bars_dict)`` must
    return SGU1DataPro.gen_dataset(19)'s table (with its 'label' column) for
    one day's event bars.  With this package's SGU2 as m2 and a float32
    StandardScaler3D, SGU2 runs on the device windows of all days at once
    (gate_units.SGU2.predict_device); any other m2 / scaler gets the host
    windows as in the reference."""
    import pandas as pd
    if sgu1_features is None:
        raise NotImplementedError("SGU1's feature table (HFTLoader.py:66-135, an xgboost input) is not "
                                  "part of this path: pass sgu1_features=callable(event_bars_dict)")
    snap_dir = os.path.join(data_root, "data", symbol, "snap")
    tick_dir = os.path.join(data_root, "data", symbol, "tick")
    days, kept = [], []
    for d in date_list:
        snap = pd.read_parquet(os.path.join(snap_dir, f"{d}.parquet"))
        tick = pd.read_parquet(os.path.join(tick_dir, f"{d}.parquet"))
        snap, tick = _filter_sort(snap, tick)
        if snap.empty:
            continue
        days.append((snap, tick))
        kept.append(d)
    ev = EventBarsGPU(days, device)
    wins = ev.windows()
    s2_all = None
    if _fused_sgu2(m2, scaler):  # every day's windows through SGU2 in one launch, scaled in the kernel
        s2_all = m2.predict_device(ev.X_all, scaler).cpu().numpy()
    s1s, s2s, n_samples, used = [], [], [], []
    for k in range(len(days)):
        df1 = sgu1_features(ev.day(k))
        n_win = int(ev.n_windows[k])
        if len(df1) == 0 or n_win == 0:
            n_samples.append(0)
            continue
        s1 = np.asarray(m1.predict(df1.drop(columns=["label"])))
        if s2_all is not None:
            s2 = s2_all[ev.win_off[k]:ev.win_off[k] + n_win]
        else:
            s2 = np.asarray(m2.predict(scaler.transform(wins[k][0].cpu().numpy()))).flatten()
        n = min(len(s1), len(s2))
        s1s.append(s1[-n:][:-1])
        s2s.append(s2[-n:][:-1])
        n_samples.append(n)
        used.append(k)
    if not used:  # the reference's np.concatenate([]) (agent_trainer.py:76)
        raise ValueError("need at least one array to concatenate")
    (mid, ask, bid, bmax, smin), _ = ev.steps(n_samples)
    return (np.concatenate(s1s), np.concatenate(s2s), mid.cpu().numpy(), ask.cpu().numpy(), bid.cpu().numpy(),
            bmax.cpu().numpy(), smin.cpu().numpy())
