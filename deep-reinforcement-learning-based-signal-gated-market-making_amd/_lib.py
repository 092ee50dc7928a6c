"""ctypes binding of libsgmm.so (the C ABI declared in include/sgmm.h).

The library is the product's only compute path.  If it is missing or cannot
load, every GPU entry point raises -- there is deliberately no CPU fallback.

torch is imported first so that libsgmm.so's libamdhip64.so.7 dependency
resolves to the HIP runtime torch already loaded (one runtime per process;
torch tensors' device pointers and streams are then valid in our calls).
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import torch  # noqa: F401  (must precede loading libsgmm.so, see module doc)

PKG_DIR = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("SGMM_LIB", PKG_DIR / "libsgmm.so"))
ABI_VERSION = 5


class SgmmError(RuntimeError):
    pass


# ----------------------------------------------------------------- structs (mirror include/sgmm.h)
class EnvParams(ctypes.Structure):
    _fields_ = [("phi", ctypes.c_double), ("tick", ctypes.c_double), ("fee", ctypes.c_double),
                ("idle_penalty", ctypes.c_double), ("i_max", ctypes.c_int32),
                ("i_min", ctypes.c_int32), ("act_scale", ctypes.c_float),
                ("adv_scale", ctypes.c_float)]


class Ticks(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in
                ("s1n", "s2n", "mid_next", "best_ask", "best_bid", "buy_max", "sell_min")]


class Episodes(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int32), ("max_len", ctypes.c_int32),
                ("total_steps", ctypes.c_int64), ("inv_min", ctypes.c_int32),
                ("inv_max", ctypes.c_int32), ("genome", ctypes.c_void_p),
                ("adv", ctypes.c_void_p), ("tick_off", ctypes.c_void_p),
                ("len", ctypes.c_void_p), ("step_off", ctypes.c_void_p),
                ("param", ctypes.c_void_p), ("order", ctypes.c_void_p)]


class GAState(ctypes.Structure):
    _fields_ = [("sigma_mm", ctypes.c_double), ("sigma_adv", ctypes.c_double),
                ("best_val", ctypes.c_double), ("last_train_f", ctypes.c_double),
                ("last_val_f", ctypes.c_double), ("no_improve", ctypes.c_int32),
                ("best_idx", ctypes.c_int32), ("adv_best_idx", ctypes.c_int32),
                ("gen", ctypes.c_int32), ("improved", ctypes.c_int32),
                ("decayed", ctypes.c_int32), ("patience", ctypes.c_int32),
                ("arrivals", ctypes.c_int32), ("decay", ctypes.c_double)]


class AskedPopulation(ctypes.Structure):
    _fields_ = [("state", ctypes.c_void_p), ("master_mm", ctypes.c_void_p), ("master_adv", ctypes.c_void_p),
                ("seed", ctypes.c_uint64), ("i0", ctypes.c_int32), ("pad_", ctypes.c_int32)]


class Populations(ctypes.Structure):
    """sgmm_populations: K GA populations advanced together (device pointers)."""
    _fields_ = [("n_pop", ctypes.c_int32), ("P", ctypes.c_int32), ("hidden", ctypes.c_int32),
                ("history_cap", ctypes.c_int32)] + \
        [(n, ctypes.c_void_p) for n in ("states", "masters_mm", "masters_adv", "best_masters", "seeds",
                                        "history", "walk_order")]


class DayStreams(ctypes.Structure):
    _fields_ = [("n_days", ctypes.c_int32), ("pad_", ctypes.c_int32), ("tick_total", ctypes.c_int64)] + \
        [(n, ctypes.c_void_p) for n in ("snap_off", "snap_time", "bid", "ask", "bidvol", "askvol",
                                        "tick_off", "tick_time", "price", "volume", "side")]


class EventBars(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("n_events", "trade_time", "ask", "bid", "p_buy_max",
                                               "p_sell_min", "v_buy_sum", "v_sell_sum", "vol_sum",
                                               "trade_count", "vwap_num")]


class GAHistory(ctypes.Structure):
    _fields_ = [("train_f", ctypes.c_double), ("val_f", ctypes.c_double),
                ("sigma_after", ctypes.c_double), ("train_trades", ctypes.c_int32),
                ("val_trades", ctypes.c_int32), ("best_idx", ctypes.c_int32),
                ("flags", ctypes.c_int32)]


assert ctypes.sizeof(EnvParams) == 48
assert ctypes.sizeof(GAState) == 80
assert ctypes.sizeof(GAHistory) == 40
assert ctypes.sizeof(Populations) == 72

_VP, _I32, _I64, _U32, _U64, _D, _SZ = (ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64,
                                        ctypes.c_uint32, ctypes.c_uint64, ctypes.c_double,
                                        ctypes.c_size_t)

# name -> (restype, argtypes); the symbol set of include/sgmm.h
SIGNATURES = {
    "sgmm_abi_version": (ctypes.c_int, []),
    "sgmm_last_error": (ctypes.c_char_p, []),
    "sgmm_env_step_batch": (ctypes.c_int, [_VP] * 17 + [_I64, _VP]),
    "sgmm_policy_forward": (ctypes.c_int, [_VP, _I64, _I32, _VP, _VP, _VP, _I64, _VP]),
    "sgmm_adversary_forward": (ctypes.c_int, [_VP, _I64, _VP, _VP, _VP, _I64, _VP]),
    "sgmm_rollout_workspace_size": (_SZ, [_I32, _I64, _I32]),
    "sgmm_rollout_workspace_bytes": (_SZ, [_I32, _I64, _I32, _I32]),
    "sgmm_rollout_fitness": (ctypes.c_int, [ctypes.POINTER(Ticks), ctypes.POINTER(Episodes), _VP,
                                            _VP, _I64, _I32, _VP, _I64, _VP, _VP, _VP, _SZ, _VP]),
    "sgmm_rollout_trace": (ctypes.c_int, [ctypes.POINTER(Ticks), ctypes.POINTER(Episodes), _VP,
                                          _VP, _I64, _I32, _VP, _I64] + [_VP] * 16),
    "sgmm_ga_ask": (ctypes.c_int, [_VP, _I64, _VP, _U32, _U64, _I32, _I32, _VP, _I64, _VP]),
    "sgmm_ga_state_init": (ctypes.c_int, [_VP, _D, _I32, _D, _VP]),
    "sgmm_ga_tell": (ctypes.c_int, [_VP, _VP, _VP, _I32, _VP, _VP, _I64, _VP, _VP, _I64, _I64,
                                    _I64, _U64, _VP, _I32, _VP]),
    "sgmm_ga_val_update": (ctypes.c_int, [_VP, _VP, _VP, _I32, _VP, _VP, _I64, _VP, _I32, _VP]),
    "sgmm_ga_step": (ctypes.c_int, [_VP, _VP, _VP, _VP, _VP, _I32, _I32, _I64, _VP, _VP, _VP, _I64, _I64, _U64,
                                    _VP, _I32, _VP, _VP, _I32, _I32, _VP]),
    "sgmm_ordered_sum": (ctypes.c_int, [_VP, _I64, ctypes.c_double, _VP, _VP]),
    "sgmm_rollout_fitness_asked": (ctypes.c_int, [ctypes.POINTER(Ticks), ctypes.POINTER(Episodes), _VP,
                                                  ctypes.POINTER(AskedPopulation), _I32, _VP, _VP, _VP,
                                                  ctypes.c_size_t, _VP]),
    "sgmm_generation": (ctypes.c_int, [ctypes.POINTER(Ticks), ctypes.POINTER(Episodes), _VP, _VP, _VP, _VP, _VP,
                                       _I32, _U64, _I32, _VP, _VP, _VP, _I32, _VP, ctypes.c_size_t, _VP]),
    "sgmm_generation_multi": (ctypes.c_int, [ctypes.POINTER(Ticks), ctypes.POINTER(Episodes), _VP,
                                             ctypes.POINTER(Populations), _VP, _VP, _VP, ctypes.c_size_t, _VP]),
    "sgmm_rollout_fitness_asked_multi": (ctypes.c_int, [ctypes.POINTER(Ticks), ctypes.POINTER(Episodes), _VP,
                                                        ctypes.POINTER(Populations), _I32, _I32, _VP, _VP, _VP,
                                                        ctypes.c_size_t, _VP]),
    "sgmm_ga_step_multi": (ctypes.c_int, [ctypes.POINTER(Populations), _VP, _VP, _VP, _VP, _I64, _I64, _I32,
                                          _I64, _VP]),
    "sgmm_generation_multi_best": (ctypes.c_int, [ctypes.POINTER(Ticks), ctypes.POINTER(Episodes),
                                                  ctypes.POINTER(Episodes), _VP, ctypes.POINTER(Populations),
                                                  _VP, _VP, _VP, _VP, _VP, ctypes.c_size_t, _VP]),
    "sgmm_validate_multi": (ctypes.c_int, [ctypes.POINTER(Ticks), ctypes.POINTER(Episodes), _VP,
                                           ctypes.POINTER(Populations), _VP, _VP, _VP, ctypes.c_size_t, _VP]),
    "sgmm_ga_tell_multi": (ctypes.c_int, [ctypes.POINTER(Populations), _VP, _VP, _I64, _I64, _I32, _I64, _VP]),
    "sgmm_event_bars_workspace_size": (ctypes.c_size_t, [_I64]),
    "sgmm_event_bars_build": (ctypes.c_int, [ctypes.POINTER(DayStreams), ctypes.POINTER(EventBars), _VP,
                                             ctypes.c_size_t, _VP]),
    "sgmm_bar_windows": (ctypes.c_int, [ctypes.POINTER(EventBars), _I32, _VP, _VP, _VP, _VP, _VP, _I64, _VP]),
    "sgmm_sgu2_forward": (ctypes.c_int, [_VP, _I32, _VP, _I64, _I32, _VP, _VP, _VP, _VP]),
    "sgmm_step_bundle": (ctypes.c_int, [ctypes.POINTER(EventBars), _I32, _VP, _VP, _VP, _I32, _VP, _VP, _VP,
                                        _VP, _VP, _VP]),
    "sgmm_plan_set": (ctypes.c_int, [_I32, _I32]),
    "sgmm_plan_get": (ctypes.c_int, [_I32]),
    "sgmm_profile_enable": (ctypes.c_int, [ctypes.c_int]),
    "sgmm_profile_read": (ctypes.c_int, [ctypes.c_int, _VP, _VP, _VP]),
}

_lib = None


def load(path: Path | None = None):
    """Load libsgmm.so and bind every symbol; raise SgmmError if impossible."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = Path(path) if path else LIB_PATH
    if not p.exists():
        raise SgmmError(f"{p} is missing: build it with `python -c 'import __graft_entry__ as g; "
                        f"g.build()'` (hipcc --offload-arch=gfx950). There is no CPU fallback.")
    L = ctypes.CDLL(str(p))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    if L.sgmm_abi_version() != ABI_VERSION:
        raise SgmmError(f"libsgmm ABI {L.sgmm_abi_version()} != {ABI_VERSION}")
    if path is None:
        _lib = L
    return L


def check(rc: int, what: str):
    if rc != 0:
        msg = _lib.sgmm_last_error().decode() if _lib is not None else ""
        raise SgmmError(f"{what} failed (rc={rc}): {msg}")


def ptr(t):
    """Raw device pointer of a torch tensor (None -> NULL)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


def stream_ptr(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def require_gpu():
    if not torch.cuda.is_available():
        raise SgmmError("no HIP device visible: the sgmm rollout path runs only on the GPU "
                        "(MI355X / gfx950); there is no CPU fallback")


def profile_enable(on: bool = True):
    load().sgmm_profile_enable(1 if on else 0)


def profile_read(max_kinds: int = 32) -> dict:
    """{kernel kind: (total_ms, launches)} since the last read (waits for events)."""
    import numpy as np
    L = load()
    names = ctypes.create_string_buffer(48 * max_kinds)
    tot = np.zeros(max_kinds, np.float64)
    cnt = np.zeros(max_kinds, np.int64)
    n = L.sgmm_profile_read(max_kinds, names, tot.ctypes.data, cnt.ctypes.data)
    check(n if n < 0 else 0, "sgmm_profile_read")
    raw = names.raw
    return {raw[48 * i:48 * i + 48].split(b"\0", 1)[0].decode(): (float(tot[i]), int(cnt[i]))
            for i in range(n)}


# launch-plan overrides (include/sgmm.h SGMM_PLAN_*): tests and A/B experiments
PLAN_KNOBS = {"policy_path": 0, "groups": 1, "lane_split": 2, "tail": 3, "four": 4, "min_eps": 5,
              "table_sp": 6, "scan_threads": 7, "reorder_weights": 8, "spill": 9, "seq_sum": 10,
              "fused_scan": 11, "lanes_scan": 12}
POLICY_PATHS = {"auto": -1, "frontier": 1, "table": 2, "valu": 3}


def plan_set(**knobs) -> dict:
    """Set launch-plan overrides (None or a negative value = the default rule);
    returns the previous values.  policy_path takes "auto" / "frontier" /
    "table" / "valu".  Applies to launches enqueued (or graphs captured) after
    the call."""
    L = load()
    prev = {}
    for k, v in knobs.items():
        if k not in PLAN_KNOBS:
            raise SgmmError(f"unknown plan knob {k!r}")
        if k == "policy_path" and isinstance(v, str):
            v = POLICY_PATHS[v]
        prev[k] = L.sgmm_plan_get(PLAN_KNOBS[k])
        check(L.sgmm_plan_set(PLAN_KNOBS[k], -1 if v is None else int(v)), "sgmm_plan_set")
    return prev


class plan:
    """Context manager: `with plan(groups=2, policy_path="frontier"): ...`"""

    def __init__(self, **knobs):
        self.knobs = knobs
        self.prev = None

    def __enter__(self):
        self.prev = plan_set(**self.knobs)
        return self

    def __exit__(self, *exc):
        plan_set(**self.prev)
        return False
