"""FPT (first-passage) limit-order matching environment.

``FTPEnv``       -- the reference's single-environment API (Env/market_env.py:3-67),
                    host-side, for the scalar loops the reference runs on CPU
                    (BASELINE config 1: one episode stepped from Python, the
                    blind-test / backtest recorder loops).  Same constructor,
                    attributes (inventory, cash, i_max, i_min), reset() and
                    step() results.
``FTPEnvBatch``  -- N environments stepped in lock-step on the GPU through
                    sgmm_env_step_batch (the batched form of the same step).

The population rollout (the hot path) does not step either of these: it runs
whole episodes inside the HIP kernels (see rollout.py / drl_engine.py).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import check, ptr, stream_ptr


class FTPEnv:
    """Match-making engine by FTP (first traversed price), market_env.py:3-67.

    A quote fills when the step's traded extreme reaches it: the bid fills if
    ``best_bid - off_b*tick >= sell_min``, the ask if
    ``best_ask + off_a*tick <= buy_max``, each subject to the inventory caps
    evaluated on the pre-step inventory.  Reward = fill PnL marked to the next
    mid, minus fees, minus ``phi * |inventory after the step|``."""

    def __init__(self, phi=0.01, tick_size=0.01, fee_rate=0.0000):
        self.fee_rate = fee_rate
        self.phi = phi
        self.tick_size = tick_size
        self.i_max, self.i_min = 2, -2
        self.inventory, self.cash = 0, 0.0

    def reset(self):
        self.inventory, self.cash = 0, 0.0
        return self.inventory, self.cash

    def step(self, action, mid_next, best_ask, best_bid, buy_max, sell_min, adv_action=None):
        da = db = 0
        if adv_action is not None:
            da, db = np.round(adv_action).astype(int)
        ask_quote = best_ask + (action[0] + da) * self.tick_size
        bid_quote = best_bid - (action[1] + db) * self.tick_size
        position = self.inventory
        bought = 1 if (position < self.i_max and bid_quote >= sell_min) else 0
        sold = 1 if (position > self.i_min and ask_quote <= buy_max) else 0
        fill_pnl, fees = 0.0, 0.0
        for filled, side, quote in ((bought, 1, bid_quote), (sold, -1, ask_quote)):
            if not filled:
                continue
            fee = quote * self.fee_rate
            self.inventory += side
            if side > 0:
                self.cash -= (quote + fee)
                fill_pnl += (mid_next - quote) - fee
            else:
                self.cash += (quote - fee)
                fill_pnl += (quote - mid_next) - fee
            fees += fee
        penalty = self.phi * abs(self.inventory)
        return fill_pnl - penalty, {
            "pnl_reward": fill_pnl,
            "inventory_reward": -penalty,
            "fee_paid": fees,
            "fill_buy": bought,
            "fill_sell": sold,
        }


class FTPEnvBatch:
    """N FPT environments on the GPU, stepped together (sgmm_env_step_batch).

    Per-environment parameters: ``phi``/``tick_size``/``fee_rate`` may be
    scalars or length-N sequences.  State lives in device tensors
    ``inventory`` (int32) and ``cash`` (float64)."""

    def __init__(self, n, phi=0.01, tick_size=0.01, fee_rate=0.0, device="cuda", i_max=2, i_min=-2):
        from .rollout import EnvConfig, params_tensor
        _lib.require_gpu()
        self.L = _lib.load()
        self.n = int(n)
        self.device = torch.device(device)
        cols = [np.broadcast_to(np.asarray(v, np.float64), (self.n,)) for v in (phi, tick_size, fee_rate)]
        cfgs = [EnvConfig(phi=float(a), tick_size=float(b), fee_rate=float(c), i_max=i_max, i_min=i_min)
                for a, b, c in zip(*cols)]
        self.params = params_tensor(cfgs, self.device)
        self.param_idx = torch.arange(self.n, dtype=torch.int32, device=self.device)
        self.reset()

    def reset(self):
        self.inventory = torch.zeros(self.n, dtype=torch.int32, device=self.device)
        self.cash = torch.zeros(self.n, dtype=torch.float64, device=self.device)
        return self.inventory, self.cash

    def step(self, action, mid_next, best_ask, best_bid, buy_max, sell_min, adv_action=None, stream=None):
        dv = self.device

        def f64(x):
            return torch.as_tensor(x, dtype=torch.float64, device=dv).expand(self.n).contiguous()

        act = torch.as_tensor(action, dtype=torch.int32, device=dv).reshape(self.n, 2).contiguous()
        adv = None if adv_action is None else \
            torch.as_tensor(np.round(np.asarray(adv_action)) if not torch.is_tensor(adv_action) else adv_action,
                            dtype=torch.int32, device=dv).reshape(self.n, 2).contiguous()
        cols = [f64(x) for x in (mid_next, best_ask, best_bid, buy_max, sell_min)]
        out = {k: torch.empty(self.n, dtype=torch.float64, device=dv)
               for k in ("reward", "pnl_reward", "inventory_reward", "fee_paid")}
        fb = torch.empty(self.n, dtype=torch.uint8, device=dv)
        fs = torch.empty(self.n, dtype=torch.uint8, device=dv)
        rc = self.L.sgmm_env_step_batch(
            ptr(self.params), ptr(self.param_idx), ptr(self.inventory), ptr(self.cash), ptr(act), ptr(adv),
            *[ptr(c) for c in cols], ptr(out["reward"]), ptr(out["pnl_reward"]),
            ptr(out["inventory_reward"]), ptr(out["fee_paid"]), ptr(fb), ptr(fs), self.n,
            stream_ptr(stream))
        check(rc, "sgmm_env_step_batch")
        info = {"pnl_reward": out["pnl_reward"], "inventory_reward": out["inventory_reward"],
                "fee_paid": out["fee_paid"], "fill_buy": fb, "fill_sell": fs}
        return out["reward"], info
