"""Device-resident rollout engine: bundles in HBM, episode batches, and the
calls into libsgmm.so's hot path.

Vocabulary (reference): a *bundle* is the 7-tuple of tick columns
(s1, s2, mid_next, best_ask, best_bid, buy_max, sell_min) that
load_signals_bundle returns (pipeline/agent_trainer.py:15-77); an *episode* is
one evaluate_individual call (Env/drl_engine.py:9-67): a genome (plus an
optional adversary genome) stepped over a bundle with (phi, tick, fee).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field

import numpy as np
import torch

from . import _lib
from ._lib import EnvParams, Episodes, Ticks, check, ptr, stream_ptr

ENV_PARAMS_DTYPE = np.dtype([("phi", "<f8"), ("tick", "<f8"), ("fee", "<f8"),
                             ("idle_penalty", "<f8"), ("i_max", "<i4"), ("i_min", "<i4"),
                             ("act_scale", "<f4"), ("adv_scale", "<f4")])
assert ENV_PARAMS_DTYPE.itemsize == ctypes.sizeof(EnvParams)

COLUMNS = ("s1n", "s2n", "mid_next", "best_ask", "best_bid", "buy_max", "sell_min")


def normalize_signals(s1, s2, train_stats):
    """State features of drl_engine.py:33-34 as float32 arrays.

    The reference evaluates ``(s[t] - m) / sd`` on numpy scalars and lets
    torch.tensor(..., dtype=float32) round the result; under NumPy >= 2 the
    vectorised expression has the same promotions (NEP 50), so each element
    equals the reference's per-step value."""
    a = (np.asarray(s1) - train_stats["s1_m"]) / train_stats["s1_s"]
    b = (np.asarray(s2) - train_stats["s2_m"]) / train_stats["s2_s"]
    return np.asarray(a).astype(np.float32), np.asarray(b).astype(np.float32)


@dataclass
class EnvConfig:
    """FTPEnv constructor arguments + evaluate_individual's constants."""
    phi: float = 0.01
    tick_size: float = 0.01
    fee_rate: float = 0.0
    idle_penalty: float = 50.0
    i_max: int = 2
    i_min: int = -2
    act_scale: float = 5.0
    adv_scale: float = 1.0

    def record(self):
        r = np.zeros((), ENV_PARAMS_DTYPE)
        r["phi"], r["tick"], r["fee"] = self.phi, self.tick_size, self.fee_rate
        r["idle_penalty"], r["i_max"], r["i_min"] = self.idle_penalty, self.i_max, self.i_min
        r["act_scale"], r["adv_scale"] = self.act_scale, self.adv_scale
        return r


def params_tensor(configs, device) -> torch.Tensor:
    recs = np.stack([c.record() for c in configs]).astype(ENV_PARAMS_DTYPE)
    return torch.from_numpy(recs.view(np.uint8).copy()).to(device)


class TickStore:
    """Concatenated SoA tick columns of several bundles, resident on device."""

    def __init__(self):
        self._parts = {c: [] for c in COLUMNS}
        self.segments = []  # (offset, length)
        self.n = 0
        self.cols = None

    def add(self, bundle, train_stats) -> int:
        """Append a bundle; returns its segment index."""
        s1, s2, mid, ask, bid, bmax, smin = bundle
        s1n, s2n = normalize_signals(s1, s2, train_stats)
        T = len(mid)
        for c, a, dt in zip(COLUMNS, (s1n, s2n, mid, ask, bid, bmax, smin),
                            (np.float32, np.float32) + (np.float64,) * 5):
            a = np.asarray(a)
            if len(a) != T:
                raise ValueError(f"bundle column {c} has length {len(a)} != {T}")
            self._parts[c].append(np.ascontiguousarray(a, dt))
        self.segments.append((self.n, T))
        self.n += T
        return len(self.segments) - 1

    def to(self, device):
        self.cols = {c: torch.from_numpy(np.concatenate(v) if v else np.zeros(0, np.float64)).to(device)
                     for c, v in self._parts.items()}
        self._parts = None
        return self

    def struct(self) -> Ticks:
        return Ticks(*[self.cols[c].data_ptr() for c in COLUMNS])


@dataclass
class EpisodeBatch:
    """Host description of a batch of episodes -> device arrays + C struct."""
    genome: np.ndarray
    tick_off: np.ndarray
    length: np.ndarray
    param: np.ndarray
    adv: np.ndarray | None = None
    inv_min: int = -2
    inv_max: int = 2
    dev: dict = field(default_factory=dict)

    def __post_init__(self):
        self.genome = np.ascontiguousarray(self.genome, np.int32)
        self.tick_off = np.ascontiguousarray(self.tick_off, np.int64)
        self.length = np.ascontiguousarray(self.length, np.int32)
        self.param = np.ascontiguousarray(self.param, np.int32)
        if self.adv is not None:
            self.adv = np.ascontiguousarray(self.adv, np.int32)
        self.step_off = np.concatenate([[0], np.cumsum(self.length.astype(np.int64))[:-1]]).astype(np.int64) \
            if len(self.length) else np.zeros(0, np.int64)
        self.total_steps = int(self.length.astype(np.int64).sum())
        self.max_len = int(self.length.max()) if len(self.length) else 0
        # longest first (stable): the frontier kernel's processing order
        self.order = np.argsort(-self.length.astype(np.int64), kind="stable").astype(np.int32)

    @property
    def n(self):
        return len(self.genome)

    def to(self, device):
        for k in ("genome", "tick_off", "length", "param", "step_off", "adv", "order"):
            v = getattr(self, k)
            self.dev[k] = None if v is None else torch.from_numpy(v).to(device)
        return self

    def struct(self) -> Episodes:
        d = self.dev
        return Episodes(self.n, self.max_len, self.total_steps, self.inv_min, self.inv_max,
                        d["genome"].data_ptr(), d["adv"].data_ptr() if d["adv"] is not None else None,
                        d["tick_off"].data_ptr(), d["length"].data_ptr(), d["step_off"].data_ptr(),
                        d["param"].data_ptr(), d["order"].data_ptr() if d.get("order") is not None else None)


class RolloutEngine:
    """Owns the workspace; enqueues sgmm_rollout_fitness / sgmm_rollout_trace."""

    def __init__(self, device="cuda"):
        _lib.require_gpu()
        self.L = _lib.load()
        self.device = torch.device(device)
        self._ws = None

    def workspace_bytes(self, eps: EpisodeBatch, arl: bool) -> int:
        nsi = eps.inv_max - eps.inv_min + 1
        return int(self.L.sgmm_rollout_workspace_bytes(eps.n, eps.total_steps, nsi, 1 if arl else 0))

    def reserve(self, eps: EpisodeBatch, arl: bool):
        """Grow the workspace for this batch now (never inside a graph capture:
        a captured launch must not see its workspace reallocated later)."""
        self.workspace(eps, arl)

    def workspace(self, eps: EpisodeBatch, arl: bool) -> torch.Tensor:
        need = self.workspace_bytes(eps, arl)
        if self._ws is None or self._ws.numel() < need:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("workspace growth during graph capture; call reserve() first")
            self._ws = torch.empty(max(need, 256), dtype=torch.uint8, device=self.device)
        return self._ws

    def fitness(self, ticks: TickStore, eps: EpisodeBatch, params: torch.Tensor, mm: torch.Tensor,
                hidden: int, adv: torch.Tensor | None = None, out=None, stream=None):
        """Fitness (f64[E]) and trades (i32[E]) of every episode; stream-ordered."""
        if out is None:
            out = (torch.empty(eps.n, dtype=torch.float64, device=self.device),
                   torch.empty(eps.n, dtype=torch.int32, device=self.device))
        ws = self.workspace(eps, adv is not None)
        tk, ep = ticks.struct(), eps.struct()
        rc = self.L.sgmm_rollout_fitness(
            ctypes.byref(tk), ctypes.byref(ep), ptr(params), ptr(mm), mm.stride(0), hidden,
            ptr(adv), adv.stride(0) if adv is not None else 0, ptr(out[0]), ptr(out[1]),
            ptr(ws), ws.numel(), stream_ptr(stream))
        check(rc, "sgmm_rollout_fitness")
        return out

    def trace(self, ticks: TickStore, eps: EpisodeBatch, params: torch.Tensor, mm: torch.Tensor,
              hidden: int, adv: torch.Tensor | None = None, stream=None):
        """Per-step trace of every episode (dict of device tensors, rows step_off[e]+t)."""
        n = eps.total_steps
        dv = self.device
        tr = {k: torch.empty(n, dtype=dt, device=dv) for k, dt in (
            ("off_a", torch.int32), ("off_b", torch.int32), ("adv_a", torch.int32),
            ("adv_b", torch.int32), ("inventory", torch.int32), ("cash", torch.float64),
            ("reward", torch.float64), ("pnl", torch.float64), ("fee_paid", torch.float64),
            ("fill_buy", torch.uint8), ("fill_sell", torch.uint8), ("raw_a", torch.float32),
            ("raw_b", torch.float32))}
        fit = torch.empty(eps.n, dtype=torch.float64, device=dv)
        trd = torch.empty(eps.n, dtype=torch.int32, device=dv)
        tk, ep = ticks.struct(), eps.struct()
        rc = self.L.sgmm_rollout_trace(
            ctypes.byref(tk), ctypes.byref(ep), ptr(params), ptr(mm), mm.stride(0), hidden,
            ptr(adv), adv.stride(0) if adv is not None else 0,
            *[ptr(tr[k]) for k in ("off_a", "off_b", "adv_a", "adv_b", "inventory", "cash",
                                   "reward", "pnl", "fee_paid", "fill_buy", "fill_sell",
                                   "raw_a", "raw_b")],
            ptr(fit), ptr(trd), stream_ptr(stream))
        check(rc, "sgmm_rollout_trace")
        return fit, trd, tr


def policy_forward(genomes: torch.Tensor, hidden: int, states: torch.Tensor,
                   genome_idx: torch.Tensor | None = None, stream=None) -> torch.Tensor:
    """Batched TradingPolicy forward on device (models/model.py:24-26)."""
    L = _lib.load()
    out = torch.empty((states.shape[0], 2), dtype=torch.float32, device=states.device)
    rc = L.sgmm_policy_forward(ptr(genomes), genomes.stride(0), hidden, ptr(genome_idx),
                               ptr(states.contiguous()), ptr(out), states.shape[0], stream_ptr(stream))
    check(rc, "sgmm_policy_forward")
    return out


def adversary_forward(genomes: torch.Tensor, states: torch.Tensor,
                      genome_idx: torch.Tensor | None = None, stream=None) -> torch.Tensor:
    """Batched AdversaryPolicy forward on device (models/model.py:49-50)."""
    L = _lib.load()
    out = torch.empty((states.shape[0], 2), dtype=torch.float32, device=states.device)
    rc = L.sgmm_adversary_forward(ptr(genomes), genomes.stride(0), ptr(genome_idx),
                                  ptr(states.contiguous()), ptr(out), states.shape[0], stream_ptr(stream))
    check(rc, "sgmm_adversary_forward")
    return out
