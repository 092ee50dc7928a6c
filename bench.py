#!/usr/bin/env python
"""Benchmark: env-steps/sec of the GA population rollout (BASELINE.json metric).

One step = one GA generation of every population on every GPU:
  ask (population from master + sigma * N(0,1), generated inside the rollout)
  -> rollout of the populations' training episodes
  -> [N > 1: one RCCL all-gather of the fitness records]
  -> tell (argmax, new master) -> validation of each population's new master
     (one episode per population, the reference's order) -> validation
     bookkeeping / sigma decay,
run through MultiDRLEngine (K populations in the same launches).  With
--val-mode fused (the default below 256 individuals per population) every
individual's validation episode runs inside the training launch instead and
the tail picks the best's (two launches per generation).
value = training env-steps (population x training ticks, all populations,
all ranks) per generation / measured seconds per generation; validation ticks
are executed but not counted.

Workloads (--config, BASELINE.json configs; synthetic SURVEY 8d ticks):
  3 (default)  GA population 512 per lambda, lambda in {1e-4, 1e-3, 5e-3, 8e-3,
               1e-2} (five populations), TradingPolicy 3->32->32->2 (the
               reference's H), one full 510300.SH trading day at event_step=1
               (4560 training ticks) + 912 validation ticks.  N > 1: weak
               scaling, every rank owns 512 individuals of each population.
  2            population 64, 3->16->16->2, 3600 + 720 ticks, phi 1e-4; weak.
  4            adversarial co-training: 256 MM + 256 adversaries paired i<->i,
               H=32, 3600 + 720 ticks; the 256 pairs split over the N ranks
               (strong).
  5            two assets (510300: tick 0.001, phi 1e-4; 688981: tick 0.01,
               phi 1e-2) x population 4096, H=32, 3600 + 720 ticks; each
               population split over the N ranks (strong).
  6, 7         not BASELINE configs: the shape the reference's own pipeline
               trains (pipeline/agent_trainer.py:136-137: DRLEngine(pop_size=50),
               H=32, ~15 training days = 3600 ticks + 720 validation ticks),
               phi 1e-4 on 510300 ticks; 7 with the adversary (USE_ARL).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Rank 0 prints one JSON line.  The CPU baseline (rank 0, N=1 only) runs BEFORE
the GPU is touched: the reference-equivalent batch-1 torch loop
(oracle/ref_loop.py) under fork Pools of 16 and 8 workers on a bounded sample
of the same workload, plus the C oracle as a "best CPU" line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "env-steps/sec (pop×ticks) at 1/2/4/8 MI355X; generations/sec vs CPU ref"
FP32_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 vector = FP32 MFMA dense peak
HBM_PEAK_GBPS = 8000.0     # MI355X_MICROARCH.md: HBM3E spec
LAMBDAS = [0.0001, 0.001, 0.005, 0.008, 0.01]

# config -> populations [(phi, tick, asset)], P (per population), H, T train, T val, ARL, scaling
CONFIGS = {
    2: dict(pops=[(0.0001, 0.001, "510300")], P=64, H=16, T=3600, Tv=720, arl=False, scaling="weak"),
    3: dict(pops=[(l, 0.001, "510300") for l in LAMBDAS], P=512, H=32, T=4560, Tv=912, arl=False,
            scaling="weak"),
    4: dict(pops=[(0.0001, 0.001, "510300")], P=256, H=32, T=3600, Tv=720, arl=True, scaling="strong"),
    5: dict(pops=[(0.0001, 0.001, "510300"), (0.01, 0.01, "688981")], P=4096, H=32, T=3600, Tv=720,
            arl=False, scaling="strong"),
    6: dict(pops=[(0.0001, 0.001, "510300")], P=50, H=32, T=3600, Tv=720, arl=False, scaling="weak"),
    7: dict(pops=[(0.0001, 0.001, "510300")], P=50, H=32, T=3600, Tv=720, arl=True, scaling="weak"),
}
BASELINE_CONFIGS = (2, 3, 4, 5)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, default=3, choices=sorted(CONFIGS))
    ap.add_argument("--pop", type=int, default=0, help="override: individuals per population (per GPU if weak)")
    ap.add_argument("--hidden", type=int, default=0, help="override: TradingPolicy hidden width")
    ap.add_argument("--ticks", type=int, default=0, help="override: training ticks")
    ap.add_argument("--val-ticks", type=int, default=-1, help="override: validation ticks")
    ap.add_argument("--profile-steps", type=int, default=0,
                    help="timed-window generations re-run eagerly and timed kernel by kernel with HIP events "
                         "(0: all of them)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-episodes", type=int, default=256,
                    help="episodes in the CPU-baseline sample (256 x 4560 ticks: ~20 core-seconds on Pool(16))")
    ap.add_argument("--pmc", default="", help="PMC traffic summary JSON (default: newest for this config)")
    ap.add_argument("--shard-of", type=int, default=1,
                    help="strong-scaled configs (4, 5): run ONE rank's shard of an N-GPU run on this GPU "
                         "(ceil(P/N) individuals per population; no exchange) and label the line '1 of N ranks'")
    ap.add_argument("--val-mode", default="auto", choices=("auto", "fused", "best"),
                    help="DRLEngine val_mode (auto: best from 256 individuals per population shard)")
    ap.add_argument("--plan", default="",
                    help="launch-plan overrides for A/B runs, e.g. 'groups=2,spill=0' (sgmm_plan_set; "
                         "knobs: " + "policy_path groups lane_split tail four min_eps table_sp scan_threads "
                         "reorder_weights spill" + "); recorded in the line's config")
    ap.add_argument("--no-walk-feedback", action="store_true", help="DRLEngine(walk_feedback=False)")
    return ap.parse_args()


def parse_plan(text):
    out = {}
    for kv in filter(None, (x.strip() for x in text.split(","))):
        k, v = kv.split("=", 1)
        out[k.strip()] = v.strip() if k.strip() == "policy_path" else int(v)
    return out


def workload_spec(args):
    c = dict(CONFIGS[args.config])
    if args.pop:
        c["P"] = args.pop
    if args.hidden:
        c["H"] = args.hidden
    if args.ticks:
        c["T"] = args.ticks
    if args.val_ticks >= 0:
        c["Tv"] = args.val_ticks
    return c


def flop_per_step(H: int) -> int:
    """Algorithmic FLOP of one env-step's policy forward: 2 * (3H + H*H + 2H)."""
    return 2 * (3 * H + H * H + 2 * H)


def bundles(spec, seed=0):
    """{asset: (train bundle, validation bundle, train_stats)}, synthetic."""
    import sgmm_pkg
    sgmm_pkg.load()
    from sgmm_amd import synthetic
    out = {}
    for j, asset in enumerate(sorted({a for _, _, a in spec["pops"]})):
        mk = synthetic.bundle_510300 if asset == "510300" else synthetic.bundle_688981
        tr = mk(spec["T"], seed=seed + 10 * j)
        va = mk(spec["Tv"], seed=seed + 10 * j + 1)
        out[asset] = (tr, va, synthetic.train_stats(tr))
    return out


def describe(spec, world, P_glob, best_val):
    pops = spec["pops"]
    H = spec["H"]
    cfg_match = {k: v for k, v in CONFIGS.items()
                 if (v["P"], v["H"], v["T"], v["Tv"], v["pops"], v["arl"]) ==
                 (spec["P"], H, spec["T"], spec["Tv"], pops, spec["arl"])}
    c = next(iter(cfg_match), None)
    head = (f"BASELINE config {c}: " if c in BASELINE_CONFIGS else
            "the reference pipeline's training shape (agent_trainer.py:136-137, not a BASELINE config): "
            if c is not None else "custom (not a BASELINE config): ")
    lam = ", ".join(f"phi={p} tick={t} {a}" for p, t, a in pops)
    return (head + f"{len(pops)} GA population(s) x {P_glob} individuals ({lam}), "
            f"TradingPolicy 3->{H}->{H}->2{' + AdversaryPolicy pairs' if spec['arl'] else ''}, synthetic ticks "
            f"({spec['T']} train + {spec['Tv']} validation: "
            f"{'the new master of each population' if best_val else 'every individual, fused'}), {world} GPU(s), "
            f"{spec['scaling']} scaling")


def cpu_baseline(spec, n_episodes):
    """Reference-equivalent CPU loop on a bounded sample of the workload,
    before any GPU use: Pool(16) (the box's CPU share for one GPU) and
    Pool(8) (the reference's hard-coded Pool(processes=8), drl_engine.py:91),
    pools started and warmed up outside the timed map; plus the C oracle."""
    import numpy as np
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle
    import ref_loop
    import sgmm_pkg
    sgmm_pkg.load()
    from sgmm_amd import synthetic
    H = spec["H"]
    phi0, tick, asset = spec["pops"][0]
    tr, _, stats = bundles(spec)[asset]
    n = max(16, n_episodes)
    pop = synthetic.population(n, H, sigma=0.05, seed=7).numpy()
    adv = synthetic.population(n, 32, sigma=0.05, seed=8).numpy() if spec["arl"] else None
    phis = np.array([spec["pops"][i % len(spec["pops"])][0] if spec["pops"][i % len(spec["pops"])][2] == asset
                     else phi0 for i in range(n)])
    steps = n * spec["T"]
    try:
        cpu_model = next(l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name"))
    except Exception:
        cpu_model = "unknown"
    pools = {}
    trades = None
    for w in (16, 8):
        w_eff = min(w, os.cpu_count() or 1)
        with ref_loop.RefPool(pop, adv, tr, phis, tick, 0.0, stats, H, workers=w_eff) as rp:
            f, t, dt = rp.map()
        trades = t
        pools[f"pool{w}"] = {"value": steps / dt, "cores": w_eff, "seconds": dt}
    # the C restatement as a "best CPU" line (same sample, OpenMP threads)
    s1n, s2n = oracle.normalize_signals(tr[0], tr[1], stats)
    ticks = (s1n, s2n) + tuple(tr[2:])
    plist = [oracle.params(phi=float(p), tick=tick) for p in phis]
    t0 = time.perf_counter()
    cf, ct = oracle.evaluate_batch(pop, H, adv, ticks, np.arange(n), np.arange(n) if adv is not None else None,
                                   np.zeros(n), np.full(n, spec["T"]), np.arange(n), plist, n_threads=16)
    dtc = time.perf_counter() - t0
    best = pools["pool16"]
    return {"value": best["value"], "unit": "env-steps/s", "cores": best["cores"], "kind": "port",
            "sample": (f"{n} training episodes of the workload ({spec['T']} ticks, H={H}, "
                       f"{'ARL pairs, ' if adv is not None else ''}phi cycling over the populations) through "
                       f"oracle/ref_loop.py (the reference's batch-1 torch loop restated, validated against "
                       f"reference fixtures) on a fork Pool, torch threads=1, pool start-up untimed"),
            "pools": pools, "os_cpu_count": os.cpu_count(), "cpu_model": cpu_model,
            "note": "Pool(16) = the CPU share of one GPU on this box (its process guard caps pools at 16); "
                    "Pool(8) = the reference's Pool(processes=8)",
            "c_oracle": {"value": steps / dtc, "cores": 16, "seconds": dtc,
                         "trades_agree_with_port": bool(np.array_equal(np.array(trades), ct))}}


def latest_pmc(path_arg, config):
    if path_arg:
        p = Path(path_arg)
    else:
        cands = sorted((ROOT / "profiles").glob(f"*pmc_traffic_c{config}.json"))
        if not cands:
            return None
        p = cands[-1]
    try:
        return json.loads(p.read_text()) | {"file": str(p.relative_to(ROOT)) if p.is_absolute() else str(p)}
    except Exception:
        return None


def latest_trace_window(config, kname, steps=None):
    """The committed rocprofv3 kernel-trace measurement of the policy kernel over
    the same command's timed window (profiles/rNN_kernel_window_cC.txt, written by
    tools/kt_window.py from `rocprofv3 --kernel-trace` of `bench.py --config C
    --steps 20`; profiles/rNN_kernel_window_cC_sK.txt for K timed generations, e.g.
    the no-flag command's 100, preferred when it matches)."""
    import re
    cands = sorted((ROOT / "profiles").glob(f"r*_kernel_window_c{config}_s{steps}.txt")) if steps else []
    if not cands:
        cands = sorted((ROOT / "profiles").glob(f"r*_kernel_window_c{config}.txt"))
    if not cands:
        return None
    fam = "k_policy_frontier" if kname == "policy_frontier" else "k_policy_table"
    for line in cands[-1].read_text().splitlines():
        m = re.search(r"window mean\s+([0-9.]+) us over (\d+) dispatches", line)
        if m and fam in line:
            return {"us": float(m.group(1)), "dispatches": int(m.group(2)), "kernel": line.split("(")[0].strip(),
                    "source": str(cands[-1].relative_to(ROOT))}
    return None


def _series(per_gen, kname, g0):
    """One kernel's per-generation time over the profiled window: first, last,
    mean, min, max (us) and the generations they cover."""
    us = [1e3 * d[kname][0] / d[kname][1] for d in per_gen if kname in d]
    if not us:
        return None
    return {"generations": [g0, g0 + len(us) - 1], "first": us[0], "last": us[-1], "mean": sum(us) / len(us),
            "min": min(us), "max": max(us)}


def make_engine(sgmm, spec, P_glob, save_dir, dist, use_graph, val_mode, seed0=1234, walk_feedback=True):
    import torch
    torch.manual_seed(seed0)
    engines = [sgmm.DRLEngine(pop_size=P_glob, phi=phi, tick_size=tick, fee_rate=0.0, use_arl=spec["arl"],
                              save_dir=save_dir, hidden_dim=spec["H"], rng="device", seed=seed0 + 17 * k,
                              val_mode=val_mode, sync_every=10**9, verbose=False, use_graph=use_graph, dist=dist,
                              walk_feedback=walk_feedback)
               for k, (phi, tick, _) in enumerate(spec["pops"])]
    return sgmm.MultiDRLEngine(engines)


def main():
    args = parse()
    spec = workload_spec(args)
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local_rank = int(os.environ.get("LOCAL_RANK", 0))
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(spec, args.cpu_episodes)  # before the GPU is initialised (fork Pool)

    import torch
    import torch.distributed as dist

    torch.cuda.set_device(local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    import sgmm_pkg
    sgmm = sgmm_pkg.load()
    from sgmm_amd import _lib
    from sgmm_amd.shard import shard_capacity
    plan = parse_plan(args.plan)
    if plan:
        _lib.plan_set(**plan)

    P, H, T, Tv = spec["P"], spec["H"], spec["T"], spec["Tv"]
    shard_of = max(1, args.shard_of)
    if shard_of > 1:
        if spec["scaling"] != "strong" or world > 1:
            raise SystemExit("--shard-of applies to the strong-scaled configs (4, 5) on one process")
        P = shard_capacity(P, shard_of)  # one rank's shard of the N-GPU run
    P_glob = P * world if spec["scaling"] == "weak" else P
    K = len(spec["pops"])
    data = bundles(spec)
    tr = [data[a][0] for _, _, a in spec["pops"]]
    va = [data[a][1] for _, _, a in spec["pops"]]
    st = [data[a][2] for _, _, a in spec["pops"]]

    def barrier():
        if world > 1:
            dist.barrier()

    tmp = tempfile.mkdtemp(prefix="sgmm_bench_")
    eng = make_engine(sgmm, spec, P_glob, tmp, None, not args.no_graph, args.val_mode,
                      walk_feedback=not args.no_walk_feedback)
    sess = eng.session(tr, va, st, generations=args.warmup + args.steps)
    sess.steps(0, args.warmup)
    sess.capture()  # graphs recorded (not run) before the timed region
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    sess.steps(args.warmup, args.steps)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    res = sess.finish()
    ms_per_step = dt / args.steps * 1e3
    value = K * P_glob * T * args.steps / dt

    # per-kernel durations over the TIMED window: the same generations re-run
    # eagerly on this rank's shard with the timed run's seeds (so the identical
    # populations), every kernel handed a pair of HIP events recorded by its own
    # dispatch on the launch stream (hipExtLaunchKernel, sgmm_profile_*); graph
    # replays launch the identical kernels.  The policy kernel gets cheaper as
    # the populations train, so its first / last / mean over the window are
    # reported and the mean is the roofline's launch time.
    n_rank = shard_capacity(P_glob, world)
    g0 = args.warmup
    n_prof = args.steps if args.profile_steps <= 0 else min(args.steps, max(args.profile_steps, 1))
    peng = make_engine(sgmm, spec, n_rank, tmp, False, False, args.val_mode,  # the timed run's seeds
                       walk_feedback=not args.no_walk_feedback)
    psess = peng.session(tr, va, st, generations=g0 + n_prof)
    for g in range(g0):
        psess.step(g)
    torch.cuda.synchronize()
    _lib.profile_read()
    _lib.profile_enable(True)
    per_gen = []
    for g in range(g0, g0 + n_prof):
        psess.step(g)
        per_gen.append(_lib.profile_read())
    _lib.profile_enable(False)
    psess.finish()
    prof = {}
    for d in per_gen:
        for k, (ms, cnt) in d.items():
            a = prof.setdefault(k, [0.0, 0])
            a[0] += ms
            a[1] += cnt
    kernels = {k: {"avg_us": 1e3 * v[0] / v[1], "launches": v[1]} for k, v in prof.items()}
    gen_kernel_us = sum(v["avg_us"] * v["launches"] for v in kernels.values()) / max(1, n_prof)

    # roofline of the policy kernel (the FP32 compute kernel of the path): the
    # frontier kernel from 768 episodes per launch (the measured crossover), the table below that
    best_val = bool(sess.best_val)
    # the training launch: training episodes (+ every validation episode when fused)
    steps_per_launch = K * n_rank * (T if best_val else T + Tv)
    fl = flop_per_step(H)
    kname = next((k for k in ("policy_frontier", "policy_table") if k in kernels), "policy_table")
    tab = kernels.get(kname)
    pmc = latest_pmc(args.pmc, args.config)
    roofline = None
    if tab:
        achieved = steps_per_launch * fl / (tab["avg_us"] * 1e-6) / 1e12
        traffic = None
        # the training launch's entry (keys carry the template: policy_table_mfma<32,5,true>; the
        # validation launch's smaller entry of the same family is not it)
        cands = [k for k in (pmc or {}).get("kernels", {}) if k.startswith(kname)]
        pk = max(cands, key=lambda k: pmc["kernels"][k].get("hbm_bytes_per_launch") or 0) if cands else None
        if pk:
            traffic = pmc["kernels"][pk].get("hbm_bytes_per_launch")
        note = ("algorithmic = one policy forward per env-step ("
                + ("training" if best_val else "training + validation") + " ticks of one launch). "
                + ("k_policy_frontier evaluates only the inventory states a chunk's paths occupy (about 1.2-1.35 per "
                   "training tick on this workload, in 16-lane MFMA tiles)" if kname.startswith("policy_frontier") else
                   "k_policy_table_v3 evaluates every inventory state (5x this work)"))
        roofline = {"bound": "mfma", "pipe": "fp32 (gfx950 f32 MFMA peak == f32 VALU peak)",
                    "kernel": ("k_policy_frontier" if kname == "policy_frontier" else
                               "k_policy_table_mfma (adversary)" if spec["arl"] else "k_policy_table_v3"),
                    "achieved": achieved, "peak": FP32_PEAK_TFLOPS,
                    "unit": "TFLOP/s", "frac": achieved / FP32_PEAK_TFLOPS, "traffic": traffic,
                    "algorithmic": {"flop_per_env_step": fl, "env_steps_per_launch": steps_per_launch,
                                    "note": note},
                    "avg_launch_us": tab["avg_us"],
                    "launch_us_over_timed_window": _series(per_gen, kname, g0)}
        tw = latest_trace_window(args.config, kname, args.steps) if shard_of == 1 else None
        if tw:
            # the same frac from the committed rocprof trace of this command (timed window)
            tw["frac"] = steps_per_launch * fl / (tw["us"] * 1e-6) / 1e12 / FP32_PEAK_TFLOPS
            tw["note"] = ("rocprofv3 --kernel-trace of `bench.py --config %d` on a previous box, dispatches of "
                          "the timed window only (tools/kt_window.py); the live frac above is this run's" % args.config)
            roofline["trace_window"] = tw
        if traffic:
            gbps = traffic / (tab["avg_us"] * 1e-6) / 1e9
            roofline["hbm"] = {"achieved_GBps": gbps, "peak_GBps": HBM_PEAK_GBPS,
                               "frac": gbps / HBM_PEAK_GBPS, "source": pmc.get("file")}
    dominant = max(kernels.items(), key=lambda kv: kv[1]["avg_us"] * kv[1]["launches"])[0] if kernels else None

    if rank == 0:
        gens_per_s = args.steps / dt
        if cpu:
            # the other half of BASELINE's metric: generations per second of the same
            # workload on the CPU path = its env-steps/s / the workload's training
            # env-steps per generation (every population, the reference's Pool loop)
            steps_per_gen = K * P_glob * T
            cpu["generations_per_s"] = cpu["value"] / steps_per_gen
            cpu["env_steps_per_generation"] = steps_per_gen
            cpu["gpu_generations_per_s"] = gens_per_s
            cpu["generations_speedup"] = gens_per_s / cpu["generations_per_s"]
        out = {
            # a shard line is ONE rank's share of a strong-scaled run: its own metric
            # name and config id, so it cannot be taken for the whole config
            "metric": METRIC if shard_of == 1 else f"{METRIC} [one rank's shard: 1 of {shard_of}]",
            "value": value, "unit": "env-steps/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_per_step,
            "higher_is_better": True, "scaling": spec["scaling"], "vs_baseline": None,
            "dtype": "f32+f64", "data": "synthetic",
            "config": {"workload": describe(spec, world, P_glob, best_val) + (
                           f"; ONE RANK'S SHARD: 1 of {shard_of} ranks (ceil(P/{shard_of}) = {P} individuals per "
                           f"population, rollout + tell on this GPU, no exchange)" if shard_of > 1 else ""),
                       "config_id": args.config if shard_of == 1 else f"{args.config}/shard-1-of-{shard_of}",
                       "shard_of": shard_of,
                       "populations": K, "population_global": P_glob, "population_per_gpu": n_rank,
                       "phis": [p for p, _, _ in spec["pops"]], "hidden": H, "ticks_train": T, "ticks_val": Tv,
                       "adversary": spec["arl"], "val_mode": "best" if best_val else "fused",
                       "parallelism": f"population shards x{world}" + (" + RCCL all-gather" if world > 1 else ""),
                       "hip_graph": bool(sess.use_graph),
                       "graph_has_exchange": bool(sess.full_graph) if world > 1 else None,
                       "graph_capture_error": getattr(sess, "capture_error", None),
                       "plan_overrides": plan or None,
                       "walk_feedback": not args.no_walk_feedback},
            "generations_per_s": gens_per_s,
            "roofline": roofline,
            "cpu_baseline": cpu,
            "speedup_vs_cpu_baseline": (value / cpu["value"]) if cpu else None,
            "kernels": kernels,
            "dominant_kernel": dominant,
            "gen_kernel_time_us": gen_kernel_us,
            "final_train_f": [float(h["train_f"][-1]) for _, h in res],
        }
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
