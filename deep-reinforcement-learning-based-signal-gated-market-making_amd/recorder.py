"""Batched backtest recorder.

The reference records a backtest one step at a time: a batch-1 policy
forward, FTPEnv.step, and a StrategyRecorder row per step
(main.py:49-96 run_drl_backtest, pipeline/agent_trainer.py:139-155 blind
test; Env/recorder.py:4-72).  Here every backtest of a request -- several
checkpoints, a phi / fee sweep, several bundles -- is ONE sgmm_rollout_trace
launch (one episode per backtest, all steps traced on device), and the rows
come back as whole columns that are assembled into the recorder's DataFrame
schema: the same columns, order, dtypes and derived columns
(StrategyRecorder.to_dataframe, Env/recorder.py:38-53), so StrategyAnalytics
and the plotting code run unchanged on the result.

Schemas:
  "backtest"  main.py:49-96 -- the record_data dict (step, mid, ask, bid,
              off_a, off_b, action, reward, inventory, cash, fee_paid,
              s1_pred, s2_pred) updated with FTPEnv.step's info
  "blind"     agent_trainer.py:139-155 -- StrategyRecorder.record's 13 columns
(pipeline/evaluator.py's record_detailed path raises KeyError('ask') in the
reference, Env/recorder.py:19-45, so it has no frame to mirror.)
"""
from __future__ import annotations

import os

import numpy as np
import torch

from .model import TradingPolicy, genome_size, hidden_from_genome
from .rollout import EnvConfig, EpisodeBatch, RolloutEngine, TickStore, params_tensor

SCHEMAS = ("backtest", "blind")


def _genome(p) -> np.ndarray:
    if isinstance(p, torch.nn.Module):
        p = p.get_weights()
    if isinstance(p, dict):  # a TradingPolicy state_dict (checkpoint)
        p = torch.cat([p[k].reshape(-1) for k in ("net.0.weight", "net.0.bias", "net.2.weight",
                                                  "net.2.bias", "net.4.weight", "net.4.bias")])
    return np.asarray(torch.as_tensor(p, dtype=torch.float32).reshape(-1).cpu(), np.float32)


def _broadcast(x, n, name):
    if name == "bundle" and isinstance(x, tuple) and len(x) == 7:  # one bundle for all
        return [x] * n
    if np.ndim(x) == 0:
        return [x] * n
    x = list(x)
    if len(x) != n:
        raise ValueError(f"{name}: {len(x)} values for {n} backtests")
    return x


def _frame(schema, cols, bundle, phi):
    """StrategyRecorder rows of one backtest -> its to_dataframe()."""
    import pandas as pd
    s1, s2, mid, ask, bid = (np.asarray(a) for a in bundle[:5])
    T = len(mid)
    off_a = cols["off_a"].astype(np.int_)   # np.round(raw * 5).astype(int)
    off_b = cols["off_b"].astype(np.int_)
    inv = cols["inventory"].astype(np.int64)  # env.inventory is a Python int
    fb = cols["fill_buy"].astype(np.int64)
    fs = cols["fill_sell"].astype(np.int64)
    inv_reward = -(phi * np.abs(inv))        # info['inventory_reward'] = -(phi * abs(inventory))
    if schema == "backtest":
        act = np.stack([off_a, off_b], axis=1)
        df = pd.DataFrame({
            "step": np.arange(T, dtype=np.int64), "mid": mid, "ask": ask, "bid": bid,
            "off_a": off_a, "off_b": off_b, "action": list(act), "reward": cols["reward"],
            "inventory": inv, "cash": cols["cash"], "fee_paid": cols["fee_paid"],
            "s1_pred": s1, "s2_pred": s2, "pnl_reward": cols["pnl"], "inventory_reward": inv_reward,
            "fill_buy": fb, "fill_sell": fs})
    elif schema == "blind":
        df = pd.DataFrame({
            "step": np.arange(T, dtype=np.int64), "mid": mid, "ask": ask, "bid": bid,
            "off_a": off_a, "off_b": off_b, "reward": cols["reward"], "inventory": inv,
            "cash": cols["cash"], "pnl_reward": cols["pnl"], "inventory_reward": inv_reward,
            "fee_paid": cols["fee_paid"], "is_trade": fb | fs})
    else:
        raise ValueError(f"schema must be one of {SCHEMAS}")
    # Env/recorder.py:45-51
    df["spread"] = df["ask"] - df["bid"]
    df["wealth"] = df["cash"] + df["inventory"] * df["mid"]
    df["cum_reward"] = df["reward"].cumsum()
    df["skew"] = df["off_b"] - df["off_a"]
    df["cum_fees"] = df["fee_paid"].cumsum()
    df["realized_pnl"] = df["cash"]
    df["unrealized_pnl"] = df["inventory"] * df["mid"]
    return df


def run_backtests(policies, bundles, train_stats, phis, fee_rates=0.0, tick_size=0.001,
                  schema="backtest", device="cuda"):
    """Backtest every (policy, bundle, phi, fee) in one device launch.

    policies: TradingPolicy modules, state_dicts or flat genomes (one hidden
    size); bundles: one 7-tuple (load_signals_bundle's) or one per backtest;
    phis / fee_rates / tick_size: scalars or one per backtest.  Returns one
    DataFrame per backtest in the recorder schema ``schema``."""
    if schema not in SCHEMAS:
        raise ValueError(f"schema must be one of {SCHEMAS}")
    genomes = [_genome(p) for p in policies]
    n = len(genomes)
    if n == 0:
        return []
    H = hidden_from_genome(genomes[0].size)
    if any(g.size != genome_size(H) for g in genomes):
        raise ValueError("all policies of one batch must share hidden_dim")
    bundles = _broadcast(bundles, n, "bundle")
    phis, fees, ticks_ = (_broadcast(v, n, k) for v, k in ((phis, "phis"), (fee_rates, "fee_rates"),
                                                          (tick_size, "tick_size")))
    dev = torch.device(device)
    ts = TickStore()
    seg_of = {}
    seg = []
    for b in bundles:
        if id(b) not in seg_of:
            seg_of[id(b)] = ts.add(b, train_stats)
        seg.append(ts.segments[seg_of[id(b)]])
    ts.to(dev)
    params = params_tensor([EnvConfig(phi=p, tick_size=t, fee_rate=f) for p, t, f in zip(phis, ticks_, fees)], dev)
    eps = EpisodeBatch(np.arange(n), [s[0] for s in seg], [s[1] for s in seg], np.arange(n)).to(dev)
    mm = torch.from_numpy(np.stack(genomes)).to(dev)
    _, _, tr = RolloutEngine(dev).trace(ts, eps, params, mm, H)
    host = {k: v.cpu().numpy() for k, v in tr.items()}
    out = []
    for e in range(n):
        a, T = int(eps.step_off[e]), int(eps.length[e])
        cols = {k: v[a:a + T] for k, v in host.items()}
        out.append(_frame(schema, cols, bundles[e], float(phis[e])))
    return out


def run_drl_backtest(symbol, method_name, weight_path, bundle, phi, fee_rate, train_stats):
    """main.py:49-96: load the checkpoint, backtest at tick 0.001, write
    output/{symbol}/{method_name}/backtest_{phi}.parquet, return the frame
    (None with a warning when the weights are missing, as the reference)."""
    if not os.path.exists(weight_path):
        print(f"Warning: Weights not found at {weight_path}")
        return None
    policy = TradingPolicy()
    policy.load_state_dict(torch.load(weight_path, weights_only=True))
    df = run_backtests([policy], bundle, train_stats, phi, fee_rate, 0.001, schema="backtest")[0]
    save_path = f"output/{symbol}/{method_name}/backtest_{phi}.parquet"
    os.makedirs(os.path.dirname(save_path), exist_ok=True)
    df.to_parquet(save_path, index=False)
    print(f"Success: {method_name} backtest completed.")
    return df


def blind_test(policy, test_bundle, train_stats, phi, tick_size, fee_rate):
    """The blind-test loop of agent_trainer.py:139-155 (StrategyRecorder.record
    rows) as one device trace; returns recorder.to_dataframe()."""
    return run_backtests([policy], test_bundle, train_stats, phi, fee_rate, tick_size, schema="blind")[0]
