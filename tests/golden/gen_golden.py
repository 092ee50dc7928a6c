"""Generate the golden fixtures under tests/golden/ from the imported reference.

Runs ONLY in the build container, where the reference is mounted read-only at
/root/reference (override with SGMM_REFERENCE).  The reference never travels:
what is committed are the small .npz fixtures this script writes (inputs and
the reference's outputs), plus this script.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py

Fixtures ("Oracle and golden vectors"):
  g1_arl_real.npz     ARL checkpoint + 510300 OOS backtest parquet (960 steps):
                      policy actions + env trace recorded by the reference.
  g1_env_replay.npz   drl/arl/glft/foic parquets replayed through FTPEnv.step
                      with the recorded actions (env-only, bit-exact).
  g2_synthetic.npz    synthetic 510300/688981-shaped episodes through the
                      reference evaluate_individual (H=32 and H=16), per-step
                      traces recorded by wrapping FTPEnv.step.
  g3_adversary.npz    adversary-active episodes (saturated adversary genomes).
  g4_ties.npz         FPT fill-test edge cases: decimal-grid ties, NaN bounds,
                      inventory caps, both-sided fills, fees.
  g5_ga.npz           NeuroEvolution ask/tell under torch.manual_seed and full
                      DRLEngine.train histories (ARL off/on) with a fork-faithful
                      serial pool.
"""
from __future__ import annotations

import contextlib
import io
import itertools
import os
import sys
import tempfile
from pathlib import Path

import numpy as np

REF = Path(os.environ.get("SGMM_REFERENCE", "/root/reference"))
OUT = Path(__file__).resolve().parent
sys.dont_write_bytecode = True
sys.path.insert(0, str(REF))

import pandas as pd  # noqa: E402
import torch  # noqa: E402

torch.set_num_threads(1)

from Env import market_env as ref_env  # noqa: E402
from Env import drl_engine as ref_engine  # noqa: E402
from models import model as ref_model  # noqa: E402

# Train stats printed by the reference run (MM_replication_Report_JiaxingWei.ipynb:578).
# The notebook ran NumPy 1.x: means are float32 scalars, std(+1e-9) float64.
NB_STATS = {
    "s1_m": np.float32(2.0911791), "s1_s": np.float64(0.3246540139184723),
    "s2_m": np.float32(0.027029233), "s2_s": np.float64(0.5160724530683288),
}


# --------------------------------------------------------------------------- helpers
class RecordingEnv(ref_env.FTPEnv):
    """Reference FTPEnv whose step() records its inputs and outputs."""
    log = None

    def step(self, action, mid_next, best_ask, best_bid, buy_max, sell_min, adv_action=None):
        a0, a1 = int(action[0]), int(action[1])
        inv_before = self.inventory
        reward, info = super().step(action, mid_next, best_ask, best_bid, buy_max, sell_min,
                                    adv_action=adv_action)
        if RecordingEnv.log is not None:
            d = (0, 0) if adv_action is None else (int(np.round(adv_action[0])), int(np.round(adv_action[1])))
            RecordingEnv.log.append((a0, a1, d[0], d[1], inv_before, self.inventory, self.cash,
                                     reward, info["pnl_reward"], info["fee_paid"],
                                     info["fill_buy"], info["fill_sell"]))
        return reward, info


TRACE_FIELDS = ("off_a", "off_b", "adv_a", "adv_b", "inv_before", "inventory", "cash", "reward",
                "pnl", "fee_paid", "fill_buy", "fill_sell")
TRACE_DT = (np.int32, np.int32, np.int32, np.int32, np.int32, np.int32, np.float64, np.float64,
            np.float64, np.float64, np.uint8, np.uint8)


def run_reference_episode(mm_w, adv_w, bundle, phi, tick, fee, stats, use_arl, hidden=32):
    """Reference evaluate_individual, unchanged, with FTPEnv.step recorded."""
    RecordingEnv.log = []
    orig_env, orig_pol = ref_engine.FTPEnv, ref_engine.TradingPolicy
    ref_engine.FTPEnv = RecordingEnv
    if hidden != 32:
        ref_engine.TradingPolicy = lambda: ref_model.TradingPolicy(hidden_dim=hidden)
    try:
        fit, trades = ref_engine.evaluate_individual(mm_w, adv_w, bundle, phi, tick, fee, stats,
                                                     use_arl=use_arl)
    finally:
        ref_engine.FTPEnv, ref_engine.TradingPolicy = orig_env, orig_pol
    log = RecordingEnv.log
    RecordingEnv.log = None
    tr = {k: np.array([r[i] for r in log], dtype=dt) for i, (k, dt) in enumerate(zip(TRACE_FIELDS, TRACE_DT))}
    return float(fit), int(trades), tr


def ref_raw_outputs(mm_w, hidden, s1, s2, stats, inv_before):
    """Raw policy outputs the reference computed at each step (batch-1 forward)."""
    pol = ref_model.TradingPolicy(hidden_dim=hidden)
    pol.set_weights(mm_w)
    raws = np.zeros((len(s1), 2), np.float32)
    with torch.no_grad():
        for t in range(len(s1)):
            st = torch.tensor([[(s1[t] - stats["s1_m"]) / stats["s1_s"],
                                (s2[t] - stats["s2_m"]) / stats["s2_s"],
                                inv_before[t] / 2.0]], dtype=torch.float32)
            raws[t] = pol.forward(st).squeeze().numpy()
    return raws


def ref_norm(s, m, sd):
    """State feature exactly as drl_engine.py:33-34 forms it (per-step scalars)."""
    return np.array([np.float32(torch.tensor([(s[t] - m) / sd], dtype=torch.float32).item())
                     for t in range(len(s))], np.float32)


def tie_margin(raw, scale=5.0):
    """min over steps of |raw*scale - (k + 1/2)|: distance to a rounding flip."""
    v = (raw.astype(np.float32) * np.float32(scale)).astype(np.float64)
    return float(np.min(np.abs(v - np.floor(v) - 0.5)))


def synth_bundle(rng, T, tick=0.001, start=3490, nan_frac=0.0, s_loc=(2.09, 0.027),
                 s_scale=(0.325, 0.516)):
    """510300.SH-shaped synthetic ticks on the decimal tick grid."""
    inv_tick = int(round(1.0 / tick))
    steps = rng.choice([-1, 0, 1], size=T + 1, p=[0.3, 0.4, 0.3])
    bid_k = start + np.cumsum(steps)
    spread = np.where(rng.random(T + 1) < 0.974, 1, 2)
    ask_k = bid_k + spread
    ask = ask_k / inv_tick
    bid = bid_k / inv_tick
    mid_next = (ask[1:] + bid[1:]) / 2
    d_sell = rng.choice([-1, 0, 1, 2], size=T, p=[0.05, 0.55, 0.30, 0.10])
    d_buy = rng.choice([-1, 0, 1, 2], size=T, p=[0.05, 0.55, 0.30, 0.10])
    buy_max = (ask_k[:T] + d_sell) / inv_tick
    sell_min = (bid_k[:T] - d_buy) / inv_tick
    if nan_frac > 0:
        buy_max[rng.random(T) < nan_frac] = np.nan
        sell_min[rng.random(T) < nan_frac] = np.nan
    s1 = rng.normal(s_loc[0], s_scale[0], T).astype(np.float32)
    s2 = rng.normal(s_loc[1], s_scale[1], T).astype(np.float32)
    return (s1, s2, mid_next.astype(np.float64), ask[:T].astype(np.float64),
            bid[:T].astype(np.float64), buy_max.astype(np.float64), sell_min.astype(np.float64))


def np2_stats(s1, s2):
    """train_stats as agent_trainer.py:126-129 computes them (under this NumPy)."""
    return {"s1_m": np.mean(s1), "s1_s": np.std(s1) + 1e-9,
            "s2_m": np.mean(s2), "s2_s": np.std(s2) + 1e-9}


def synth_bounds_from_fills(mid, ask, bid, off_a, off_b, fill_buy, fill_sell, tick):
    """On-grid buy_max/sell_min that reproduce recorded fills (1 tick margin)."""
    inv_tick = int(round(1.0 / tick))
    ask_k = np.round(ask * inv_tick).astype(np.int64)
    bid_k = np.round(bid * inv_tick).astype(np.int64)
    qa = ask_k + off_a
    qb = bid_k - off_b
    buy_max = np.where(fill_sell == 1, qa + 1, qa - 1) / inv_tick
    sell_min = np.where(fill_buy == 1, qb - 1, qb + 1) / inv_tick
    return buy_max.astype(np.float64), sell_min.astype(np.float64)


# --------------------------------------------------------------------------- G1
def gen_g1():
    par = REF / "output" / "510300"
    out = {}
    replay = {}
    for m in ("arl", "drl", "glft", "foic"):
        df = pd.read_parquet(par / m / "backtest_0.0001.parquet")
        off_a = df["off_a"].to_numpy(np.int64)
        off_b = df["off_b"].to_numpy(np.int64)
        mid = df["mid"].to_numpy(np.float64)
        ask = df["ask"].to_numpy(np.float64)
        bid = df["bid"].to_numpy(np.float64)
        fb = df["fill_buy"].to_numpy(np.int64)
        fs = df["fill_sell"].to_numpy(np.int64)
        bmax, smin = synth_bounds_from_fills(mid, ask, bid, off_a, off_b, fb, fs, 0.001)
        # env-only replay through the reference step with the recorded actions
        env = ref_env.FTPEnv(phi=0.0001, tick_size=0.001, fee_rate=0.0)
        rec = []
        for t in range(len(mid)):
            r, info = env.step(np.array([off_a[t], off_b[t]]), mid[t], ask[t], bid[t], bmax[t], smin[t])
            rec.append((env.inventory, env.cash, r, info["pnl_reward"], info["inventory_reward"],
                        info["fee_paid"], info["fill_buy"], info["fill_sell"]))
        rec = list(zip(*rec))
        inv_r = np.array(rec[0], np.int32)
        assert np.array_equal(inv_r, df["inventory"].to_numpy()), m
        assert np.array_equal(np.array(rec[1]), df["cash"].to_numpy()), m
        assert np.array_equal(np.array(rec[2]), df["reward"].to_numpy()), m
        replay[m] = dict(
            off_a=off_a.astype(np.int32), off_b=off_b.astype(np.int32), mid=mid, ask=ask, bid=bid,
            buy_max=bmax, sell_min=smin, inventory=inv_r, cash=np.array(rec[1]),
            reward=np.array(rec[2]), pnl=np.array(rec[3]), inv_reward=np.array(rec[4]),
            fee_paid=np.array(rec[5]), fill_buy=np.array(rec[6], np.uint8),
            fill_sell=np.array(rec[7], np.uint8),
            s1_pred=df["s1_pred"].to_numpy(np.float32), s2_pred=df["s2_pred"].to_numpy(np.float32))
        if m == "arl":
            sd = torch.load(REF / "checkpoints/510300/with_adv/agent_best_val_0.0001.pth", weights_only=True)
            pol = ref_model.TradingPolicy()
            pol.load_state_dict(sd)
            genome = pol.get_weights().numpy().astype(np.float32)
            s1 = replay[m]["s1_pred"]
            s2 = replay[m]["s2_pred"]
            inv_before = np.concatenate([[0], inv_r[:-1]]).astype(np.int32)
            raws = ref_raw_outputs(torch.from_numpy(genome), 32, s1, s2, NB_STATS, inv_before)
            acts = np.round(raws * 5.0).astype(np.int64)
            assert np.array_equal(acts[:, 0], off_a) and np.array_equal(acts[:, 1], off_b)
            # and the full reference loop (policy + env) on the synthesised bounds
            bundle = (s1, s2, mid, ask, bid, bmax, smin)
            fit, trades, tr = run_reference_episode(torch.from_numpy(genome), None, bundle, 0.0001,
                                                    0.001, 0.0, NB_STATS, False)
            assert np.array_equal(tr["inventory"], inv_r)
            out = dict(genome=genome, s1_pred=s1, s2_pred=s2, mid=mid, ask=ask, bid=bid,
                       buy_max=bmax, sell_min=smin,
                       s1n=ref_norm(s1, NB_STATS["s1_m"], NB_STATS["s1_s"]),
                       s2n=ref_norm(s2, NB_STATS["s2_m"], NB_STATS["s2_s"]),
                       stats=np.array([NB_STATS["s1_m"], NB_STATS["s1_s"], NB_STATS["s2_m"],
                                       NB_STATS["s2_s"]], np.float64),
                       raw=raws, off_a=off_a.astype(np.int32), off_b=off_b.astype(np.int32),
                       inventory=inv_r, cash=replay[m]["cash"], reward=replay[m]["reward"],
                       fill_buy=replay[m]["fill_buy"], fill_sell=replay[m]["fill_sell"],
                       fitness=np.float64(fit), trades=np.int32(trades),
                       tie_margin=np.float64(tie_margin(raws)))
    np.savez_compressed(OUT / "g1_arl_real.npz", **out)
    flat = {f"{m}__{k}": v for m, d in replay.items() for k, v in d.items()}
    np.savez_compressed(OUT / "g1_env_replay.npz", **flat)
    print("g1: ok  fitness=%.6f trades=%d tie_margin=%.2e" % (out["fitness"], out["trades"], out["tie_margin"]))


# --------------------------------------------------------------------------- G2 / G3
def make_genomes(seed, n, hidden, sigma):
    torch.manual_seed(seed)
    master = ref_model.TradingPolicy(hidden_dim=hidden).get_weights()
    return [master + torch.randn_like(master) * sigma for _ in range(n)]


def gen_episodes(name, cases):
    """cases: list of dicts -> stacked fixture of episodes with per-step traces."""
    recs = []
    for c in cases:
        rng = np.random.default_rng(c["seed"])
        tick = c["tick"]
        start = 3490 if tick == 0.001 else 4500
        bundle = synth_bundle(rng, c["T"], tick=tick, start=start, nan_frac=c.get("nan", 0.0))
        stats = np2_stats(bundle[0], bundle[1]) if c.get("stats", "np2") == "np2" else NB_STATS
        mm = make_genomes(1000 + c["seed"], 1, c["H"], c["sigma"])[0]
        adv = None
        if c["arl"]:
            adv = make_genomes(2000 + c["seed"], 1, 32, c.get("adv_sigma", 0.05))[0] * c.get("adv_gain", 1.0)
        fit, trades, tr = run_reference_episode(mm, adv, bundle, c["phi"], tick, c["fee"], stats,
                                                c["arl"], hidden=c["H"])
        raws = ref_raw_outputs(mm, c["H"], bundle[0], bundle[1], stats, tr["inv_before"])
        recs.append(dict(case=c, bundle=bundle, stats=stats, mm=mm.numpy(),
                         adv=None if adv is None else adv.numpy(), fit=fit, trades=trades, tr=tr,
                         raw=raws, margin=tie_margin(raws)))
    # pack ragged episodes into concatenated arrays
    offs = np.cumsum([0] + [len(r["bundle"][2]) for r in recs]).astype(np.int64)
    o = {"ep_off": offs[:-1], "ep_len": np.diff(offs)}
    for i, k in enumerate(("s1", "s2", "mid", "ask", "bid", "buy_max", "sell_min")):
        o[k] = np.concatenate([r["bundle"][i] for r in recs])
    o["s1n"] = np.concatenate([ref_norm(r["bundle"][0], r["stats"]["s1_m"], r["stats"]["s1_s"]) for r in recs])
    o["s2n"] = np.concatenate([ref_norm(r["bundle"][1], r["stats"]["s2_m"], r["stats"]["s2_s"]) for r in recs])
    o["stats"] = np.array([[float(r["stats"][k]) for k in ("s1_m", "s1_s", "s2_m", "s2_s")] for r in recs])
    o["stats_f32_mean"] = np.array([[np.float32(r["stats"]["s1_m"]), np.float32(r["stats"]["s2_m"])] for r in recs], np.float32)
    o["stats_nb"] = np.array([r["case"].get("stats", "np2") == "nb" for r in recs], np.uint8)
    o["H"] = np.array([r["case"]["H"] for r in recs], np.int32)
    o["phi"] = np.array([r["case"]["phi"] for r in recs])
    o["tick"] = np.array([r["case"]["tick"] for r in recs])
    o["fee"] = np.array([r["case"]["fee"] for r in recs])
    o["arl"] = np.array([r["case"]["arl"] for r in recs], np.uint8)
    o["fitness"] = np.array([r["fit"] for r in recs])
    o["trades"] = np.array([r["trades"] for r in recs], np.int32)
    o["tie_margin"] = np.array([r["margin"] for r in recs])
    gmax = max(r["mm"].size for r in recs)
    o["mm"] = np.stack([np.pad(r["mm"], (0, gmax - r["mm"].size)) for r in recs]).astype(np.float32)
    o["adv"] = np.stack([r["adv"] if r["adv"] is not None else np.zeros(1250, np.float32) for r in recs]).astype(np.float32)
    o["raw"] = np.concatenate([r["raw"] for r in recs])
    for k in TRACE_FIELDS:
        o["tr_" + k] = np.concatenate([r["tr"][k] for r in recs])
    np.savez_compressed(OUT / name, **o)
    print("%s: %d episodes, %d steps, min tie margin %.2e" % (name, len(recs), offs[-1], o["tie_margin"].min()))


def gen_g2():
    cases = []
    for seed, (H, T, arl, phi, fee, tick, sigma, nan) in enumerate(itertools.product(
            (32, 16), (240,), (False, True), (0.0001, 0.01), (0.0, 3e-5), (0.001,), (0.05,), (0.0,))):
        cases.append(dict(seed=seed, H=H, T=T, arl=arl, phi=phi, fee=fee, tick=tick, sigma=sigma, nan=nan))
    # longer / wider-variance / 688981-shaped / NaN-bound episodes
    cases += [
        dict(seed=100, H=32, T=720, arl=False, phi=0.001, fee=0.0, tick=0.001, sigma=0.3),
        dict(seed=101, H=16, T=720, arl=False, phi=0.0001, fee=0.0, tick=0.001, sigma=0.5),
        dict(seed=102, H=32, T=480, arl=False, phi=0.01, fee=0.0, tick=0.01, sigma=0.2),
        dict(seed=103, H=32, T=480, arl=True, phi=0.005, fee=3e-4, tick=0.01, sigma=0.2),
        dict(seed=104, H=32, T=480, arl=False, phi=0.0001, fee=0.0, tick=0.001, sigma=0.2, nan=0.02),
        dict(seed=105, H=16, T=240, arl=False, phi=0.0001, fee=0.0, tick=0.001, sigma=0.05, stats="nb"),
        dict(seed=106, H=32, T=240, arl=False, phi=0.0001, fee=0.0, tick=0.001, sigma=8.0),  # idle policy likely
    ]
    gen_episodes("g2_synthetic.npz", cases)


def gen_g3():
    cases = []
    for seed in range(6):
        cases.append(dict(seed=200 + seed, H=32 if seed % 2 == 0 else 16, T=300, arl=True,
                          phi=(0.0001, 0.001, 0.01)[seed % 3], fee=(0.0, 3e-5)[seed % 2],
                          tick=0.001, sigma=0.1, adv_sigma=0.5, adv_gain=50.0))
    gen_episodes("g3_adversary.npz", cases)


# --------------------------------------------------------------------------- G4
def gen_g4():
    """Scripted FTPEnv.step sequences hitting the fill-test edge cases."""
    rng = np.random.default_rng(7)
    rows = []
    for tick, base in ((0.001, 3490), (0.01, 4500), (0.001, 999)):
        inv_tick = int(round(1.0 / tick))
        for fee in (0.0, 3e-5):
            env = ref_env.FTPEnv(phi=0.003, tick_size=tick, fee_rate=fee)
            for t in range(400):
                bk = base + int(rng.integers(-40, 40))
                ak = bk + int(rng.choice([1, 2]))
                oa, ob = int(rng.integers(-5, 11)), int(rng.integers(-5, 11))
                adv = None if rng.random() < 0.5 else np.array([int(rng.integers(-1, 2)), int(rng.integers(-1, 2))])
                mode = rng.integers(0, 5)
                # decimal-grid value of the quote: the tie the fp64 quote may miss
                qa_k = ak + oa + (0 if adv is None else adv[0])
                qb_k = bk - ob + (0 if adv is None else -adv[1])
                if mode == 0:      # exact decimal ties
                    bmax, smin = qa_k / inv_tick, qb_k / inv_tick
                elif mode == 1:    # NaN bounds
                    bmax, smin = (np.nan, qb_k / inv_tick) if rng.random() < 0.5 else (qa_k / inv_tick, np.nan)
                elif mode == 2:    # always fill both sides (caps decide)
                    bmax, smin = (qa_k + 5) / inv_tick, (qb_k - 5) / inv_tick
                else:              # random near-tie
                    bmax = (qa_k + int(rng.integers(-1, 2))) / inv_tick
                    smin = (qb_k + int(rng.integers(-1, 2))) / inv_tick
                mid = (ak + bk + int(rng.integers(-2, 3))) / 2 / inv_tick
                inv0, cash0 = env.inventory, env.cash
                r, info = env.step(np.array([oa, ob]), mid, ak / inv_tick, bk / inv_tick, bmax, smin,
                                   adv_action=adv)
                rows.append((tick, fee, 0.003, oa, ob, 0 if adv is None else 1,
                             0 if adv is None else adv[0], 0 if adv is None else adv[1],
                             mid, ak / inv_tick, bk / inv_tick, bmax, smin, inv0, cash0,
                             env.inventory, env.cash, r, info["pnl_reward"], info["inventory_reward"],
                             info["fee_paid"], info["fill_buy"], info["fill_sell"]))
    cols = ("tick", "fee", "phi", "off_a", "off_b", "has_adv", "adv_a", "adv_b", "mid", "ask", "bid",
            "buy_max", "sell_min", "inv_before", "cash_before", "inventory", "cash", "reward", "pnl",
            "inv_reward", "fee_paid", "fill_buy", "fill_sell")
    ints = {"off_a", "off_b", "has_adv", "adv_a", "adv_b", "inv_before", "inventory", "fill_buy", "fill_sell"}
    o = {c: np.array([r[i] for r in rows], np.int32 if c in ints else np.float64) for i, c in enumerate(cols)}
    # how many decimal-grid ties the fp64 quote arithmetic breaks (documentation)
    np.savez_compressed(OUT / "g4_ties.npz", **o)
    print("g4: %d steps, fills buy=%d sell=%d" % (len(rows), o["fill_buy"].sum(), o["fill_sell"].sum()))


# --------------------------------------------------------------------------- G5
class ForkFaithfulPool:
    """Serial stand-in for multiprocessing.Pool that keeps fork semantics for the
    parent's torch RNG: each task runs with (and then discards) a copy of the
    parent's generator state, as a forked worker would."""

    def __init__(self, processes=None):
        pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False

    def starmap(self, fn, iterable):
        out = []
        for args in iterable:
            st = torch.get_rng_state()
            out.append(fn(*args))
            torch.set_rng_state(st)
        return out


def gen_g5():
    o = {}
    # ask under a fixed seed
    torch.manual_seed(123)
    ne = ref_model.NeuroEvolution(population_size=4, sigma=0.05)
    o["ask_master"] = ne.master_policy.get_weights().numpy()
    pop = ne.ask()
    o["ask_pop"] = torch.stack(pop).numpy()
    # tell: first index of the max (np.argmax)
    fit = [0.5, 2.0, -1.0, 2.0]
    best = ne.tell(pop, fit)
    o["tell_fit"] = np.array(fit)
    o["tell_best"] = np.float64(best)
    o["tell_master"] = ne.master_policy.get_weights().numpy()
    # full training runs
    ref_engine.Pool = ForkFaithfulPool
    for arl in (False, True):
        rng = np.random.default_rng(55 + arl)
        train = synth_bundle(rng, 200)
        val = synth_bundle(rng, 60)
        stats = np2_stats(train[0], train[1])
        with tempfile.TemporaryDirectory() as td:
            torch.manual_seed(2024 + arl)
            eng = ref_engine.DRLEngine(pop_size=6, sigma=0.05, phi=0.001, tick_size=0.001,
                                       use_arl=arl, save_dir=td)
            buf = io.StringIO()
            with contextlib.redirect_stdout(buf):
                pol, hist = eng.train(train, val, stats, generations=20, output_prefix="agent")
            ck = torch.load(os.path.join(td, "agent_best_val_0.001.pth"), weights_only=True)
        tag = "arl" if arl else "drl"
        for i, k in enumerate(("s1", "s2", "mid", "ask", "bid", "buy_max", "sell_min")):
            o[f"{tag}_train_{k}"] = train[i]
            o[f"{tag}_val_{k}"] = val[i]
        o[f"{tag}_stats"] = np.array([stats[k] for k in ("s1_m", "s1_s", "s2_m", "s2_s")], np.float32)
        assert all(isinstance(stats[k], np.float32) for k in stats)
        for k, v in hist.items():
            o[f"{tag}_hist_{k}"] = np.array(v, np.float64)
        o[f"{tag}_final_master"] = pol.get_weights().numpy()
        o[f"{tag}_ckpt"] = torch.cat([ck[k].reshape(-1) for k in ck]).numpy()
        o[f"{tag}_stdout"] = np.array(buf.getvalue())
        o[f"{tag}_seed"] = np.int64(2024 + arl)
        print("g5 %s: train_f %s" % (tag, np.round(o[f"{tag}_hist_train_f"], 4)))
    np.savez_compressed(OUT / "g5_ga.npz", **o)


if __name__ == "__main__":
    which = sys.argv[1:] or ["g1", "g2", "g3", "g4", "g5"]
    for w in which:
        globals()["gen_" + w]()
