"""CPU oracle for the population-rollout hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg import this module, and only as the checker (or as the timed CPU baseline).
The product package never imports it; its GPU path fails loudly instead of
falling back here.

Two restatements live here:

* ``liboracle.so`` (``sgmm_oracle.c``): scalar C restatement of
  ``FTPEnv.step`` (Env/market_env.py:22-67), ``TradingPolicy`` /
  ``AdversaryPolicy`` forward (models/model.py:5-57) and
  ``evaluate_individual`` (Env/drl_engine.py:9-67), in the canonical fp32
  order the HIP kernels use.  Used to check the GPU results bit for bit.
* ``normalize_signals``: the state features of drl_engine.py:33-34.

Parity of the oracle itself is pinned against golden vectors produced by the
imported reference (tests/golden/gen_golden.py): per-step actions,
inventories, fills, cash and rewards ("Oracle").
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
_LIB_PATH = _HERE / "_build" / "liboracle.so"
_lib = None


class OrcParams(ctypes.Structure):
    _fields_ = [
        ("phi", ctypes.c_double),
        ("tick", ctypes.c_double),
        ("fee", ctypes.c_double),
        ("idle_penalty", ctypes.c_double),
        ("i_max", ctypes.c_int32),
        ("i_min", ctypes.c_int32),
        ("act_scale", ctypes.c_float),
        ("adv_scale", ctypes.c_float),
    ]


class OrcTrace(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in (
        "off_a", "off_b", "adv_a", "adv_b", "inventory", "cash", "reward", "pnl",
        "fee_paid", "fill_buy", "fill_sell", "raw_a", "raw_b")]


def build() -> Path:
    """Compile liboracle.so with the committed Makefile (gcc)."""
    subprocess.run(["make", "-s", "-C", str(_HERE)], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not _LIB_PATH.exists():
            build()
        L = ctypes.CDLL(str(_LIB_PATH))
        d, f, i32, i64, vp = (ctypes.c_double, ctypes.c_float, ctypes.c_int32,
                              ctypes.c_int64, ctypes.c_void_p)
        L.orc_env_step.restype = ctypes.c_int
        L.orc_env_step.argtypes = [ctypes.POINTER(OrcParams), vp, vp, i32, i32, ctypes.c_int,
                                   i32, i32, d, d, d, d, d, vp, vp]
        L.orc_policy_forward.restype = None
        L.orc_policy_forward.argtypes = [vp, ctypes.c_int, vp, vp]
        L.orc_adversary_forward.restype = None
        L.orc_adversary_forward.argtypes = [vp, vp, vp]
        L.orc_evaluate.restype = d
        L.orc_evaluate.argtypes = [vp, ctypes.c_int, vp, vp, vp, vp, vp, vp, vp, vp, i64,
                                   ctypes.POINTER(OrcParams), vp, ctypes.POINTER(OrcTrace)]
        L.orc_evaluate_batch.restype = None
        L.orc_evaluate_batch.argtypes = [vp, ctypes.c_int, i64, vp, i64, vp, vp, vp, vp, vp, vp, vp,
                                         i32, vp, vp, vp, vp, vp, ctypes.POINTER(OrcParams),
                                         vp, vp, ctypes.c_int]
        _lib = L
    return _lib


def params(phi=0.01, tick=0.01, fee=0.0, idle_penalty=50.0, i_max=2, i_min=-2,
           act_scale=5.0, adv_scale=1.0) -> OrcParams:
    return OrcParams(phi, tick, fee, idle_penalty, i_max, i_min, act_scale, adv_scale)


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def normalize_signals(s1, s2, train_stats):
    """State features of drl_engine.py:33-34: float32((s - m) / sd).

    Element-wise numpy with the reference's own scalar types (NumPy >= 2 gives
    vectorised expressions the same promotion as the reference's per-step
    scalar expression)."""
    s1 = np.asarray(s1)
    s2 = np.asarray(s2)
    a = (s1 - train_stats["s1_m"]) / train_stats["s1_s"]
    b = (s2 - train_stats["s2_m"]) / train_stats["s2_s"]
    return np.asarray(a).astype(np.float32), np.asarray(b).astype(np.float32)


def env_step(p: OrcParams, inv: int, cash: float, off_a: int, off_b: int, adv=None,
             mid=0.0, ask=0.0, bid=0.0, bmax=0.0, smin=0.0):
    """One FTPEnv.step. Returns (inv, cash, reward, pnl, inv_reward, fee, fill_buy, fill_sell)."""
    iv = np.array([inv], np.int32)
    cs = np.array([cash], np.float64)
    o4 = np.zeros(4, np.float64)
    fl = np.zeros(2, np.int32)
    has = adv is not None
    aa, ab = (int(adv[0]), int(adv[1])) if has else (0, 0)
    lib().orc_env_step(ctypes.byref(p), _p(iv), _p(cs), int(off_a), int(off_b), int(has), aa, ab,
                       float(mid), float(ask), float(bid), float(bmax), float(smin), _p(o4), _p(fl))
    return int(iv[0]), float(cs[0]), o4[0], o4[1], o4[2], o4[3], int(fl[0]), int(fl[1])


def policy_forward(genome, H, x):
    g = np.ascontiguousarray(genome, np.float32)
    xx = np.ascontiguousarray(x, np.float32)
    out = np.zeros(2, np.float32)
    lib().orc_policy_forward(_p(g), int(H), _p(xx), _p(out))
    return out


def adversary_forward(genome, x):
    g = np.ascontiguousarray(genome, np.float32)
    xx = np.ascontiguousarray(x, np.float32)
    out = np.zeros(2, np.float32)
    lib().orc_adversary_forward(_p(g), _p(xx), _p(out))
    return out


def evaluate(mm, H, adv, s1n, s2n, mid, ask, bid, bmax, smin, p: OrcParams, trace=False):
    """evaluate_individual on pre-normalised signals.

    Returns (fitness, trades) or (fitness, trades, trace_dict)."""
    T = len(mid)
    mm = np.ascontiguousarray(mm, np.float32)
    adv = None if adv is None else np.ascontiguousarray(adv, np.float32)
    arrs = [np.ascontiguousarray(a, dt) for a, dt in
            ((s1n, np.float32), (s2n, np.float32), (mid, np.float64), (ask, np.float64),
             (bid, np.float64), (bmax, np.float64), (smin, np.float64))]
    trades = np.zeros(1, np.int32)
    tr = None
    out = None
    if trace:
        out = {
            "off_a": np.zeros(T, np.int32), "off_b": np.zeros(T, np.int32),
            "adv_a": np.zeros(T, np.int32), "adv_b": np.zeros(T, np.int32),
            "inventory": np.zeros(T, np.int32), "cash": np.zeros(T, np.float64),
            "reward": np.zeros(T, np.float64), "pnl": np.zeros(T, np.float64),
            "fee_paid": np.zeros(T, np.float64), "fill_buy": np.zeros(T, np.uint8),
            "fill_sell": np.zeros(T, np.uint8), "raw_a": np.zeros(T, np.float32),
            "raw_b": np.zeros(T, np.float32),
        }
        tr = OrcTrace(**{k: v.ctypes.data for k, v in out.items()})
    fit = lib().orc_evaluate(_p(mm), int(H), _p(adv), *[_p(a) for a in arrs], int(T),
                             ctypes.byref(p), _p(trades), ctypes.byref(tr) if tr else None)
    if trace:
        return fit, int(trades[0]), out
    return fit, int(trades[0])


def evaluate_batch(mm, H, adv, ticks, ep_genome, ep_adv, ep_off, ep_len, ep_param, param_list,
                   n_threads=1):
    """Batch of episodes over concatenated tick arrays.

    ticks = (s1n, s2n, mid, ask, bid, bmax, smin); returns (fitness f64[E], trades i32[E])."""
    mm = np.ascontiguousarray(mm, np.float32)
    G = mm.shape[1]
    adv_arr = None if adv is None else np.ascontiguousarray(adv, np.float32)
    Ga = 0 if adv_arr is None else adv_arr.shape[1]
    tk = [np.ascontiguousarray(a, dt) for a, dt in zip(
        ticks, (np.float32, np.float32) + (np.float64,) * 5)]
    E = len(ep_genome)
    eg = np.ascontiguousarray(ep_genome, np.int32)
    ea = np.ascontiguousarray(ep_adv if ep_adv is not None else -np.ones(E), np.int32)
    eo = np.ascontiguousarray(ep_off, np.int64)
    el = np.ascontiguousarray(ep_len, np.int64)
    ep = np.ascontiguousarray(ep_param, np.int32)
    P = (OrcParams * len(param_list))(*param_list)
    fit = np.zeros(E, np.float64)
    trd = np.zeros(E, np.int32)
    lib().orc_evaluate_batch(_p(mm), int(H), int(G), _p(adv_arr), int(Ga), *[_p(a) for a in tk],
                             int(E), _p(eg), _p(ea), _p(eo), _p(el), _p(ep), P, _p(fit), _p(trd),
                             int(n_threads))
    return fit, trd


if os.environ.get("SGMM_ORACLE_AUTOBUILD", "1") == "1" and not _LIB_PATH.exists():
    try:
        build()
    except Exception:  # pragma: no cover - surfaced when lib() is called
        pass
