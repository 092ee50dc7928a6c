"""Rank bodies for the multi-process shard tests (importable by spawned
children; not a test module)."""
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent


def _setup(rank, world, port, backend="gloo"):
    sys.path[:0] = [str(ROOT), str(ROOT / "oracle"), str(ROOT / "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group(backend, rank=rank, world_size=world)
    import sgmm_pkg
    sgmm_pkg.load()
    return dist


def workload(P, T=300, Tv=120, H=16):
    import sgmm_pkg
    sg = sgmm_pkg.load()
    from sgmm_amd import synthetic
    tr = synthetic.bundle_510300(T, seed=0)
    va = synthetic.bundle_510300(Tv, seed=1)
    st = synthetic.train_stats(tr)
    pop = synthetic.population(P, H, sigma=0.5, seed=3).numpy()
    return sg, tr, va, st, pop


def oracle_fitness(pop, bundle, st, H, idx):
    import oracle as orc
    s1n, s2n = orc.normalize_signals(bundle[0], bundle[1], st)
    p = orc.params(phi=0.0005, tick=0.001)
    f = np.zeros(len(idx)); t = np.zeros(len(idx), np.int32)
    for k, i in enumerate(idx):
        f[k], t[k] = orc.evaluate(pop[i], H, None, s1n, s2n, *bundle[2:], p)
    return f, t


def records_rank(rank, world, port, P, outdir):
    """Each rank evaluates its shard (oracle), writes its record, all-gathers
    with gloo and saves the gathered bytes plus the decoded population."""
    dist = _setup(rank, world, port)
    try:
        from sgmm_amd.shard import FitnessRecords, shard_bounds
        _, tr, va, st, pop = workload(P)
        i0, i1 = shard_bounds(P, rank, world)
        rec = FitnessRecords(P, world, "cpu")
        idx = list(range(i0, i1))
        if idx:
            f, t = oracle_fitness(pop, tr, st, 16, idx)
            vf, vt = oracle_fitness(pop, va, st, 16, idx)
            n = i1 - i0
            import torch
            rec.train[0][:n] = torch.from_numpy(f)
            rec.train[1][:n] = torch.from_numpy(t)
            rec.val[0][:n] = torch.from_numpy(vf)
            rec.val[1][:n] = torch.from_numpy(vt)
        rec.all_gather()
        pf, pt, pvf, pvt = (x.numpy() for x in rec.population())
        np.savez(os.path.join(outdir, f"r{rank}.npz"), gathered=rec.gathered.numpy(), n=rec.n,
                 pf=pf, pt=pt, pvf=pvf, pvt=pvt)
    finally:
        dist.destroy_process_group()


MULTI_POPS = [(0.0001, 0.001, 0), (0.005, 0.001, 0), (0.01, 0.01, 1)]  # (phi, tick, asset) per population


def multi_workload():
    """Per-population (train, val, stats) lists: two assets with their own
    tick sizes and lengths, as tests/test_gpu_multi.py."""
    from sgmm_amd import synthetic
    a_tr, a_va = synthetic.bundle_510300(600, seed=10), synthetic.bundle_510300(150, seed=11)
    b_tr, b_va = synthetic.bundle_688981(520, seed=12), synthetic.bundle_688981(170, seed=13)
    assets = ((a_tr, a_va, synthetic.train_stats(a_tr)), (b_tr, b_va, synthetic.train_stats(b_tr)))
    return ([assets[a][j] for _, _, a in MULTI_POPS] for j in range(3))


def multi_engines(sg, P, arl, save_dir, val_mode, dist=None):
    import torch
    engines = []
    for k, (phi, tick, _) in enumerate(MULTI_POPS):
        torch.manual_seed(100 + k)  # the initial masters come from the torch generator
        engines.append(sg.DRLEngine(pop_size=P, phi=phi, tick_size=tick, use_arl=arl, save_dir=save_dir,
                                    hidden_dim=16, rng="device", seed=1000 + 7 * k, val_mode=val_mode,
                                    sync_every=5, patience=3, verbose=False, dist=dist))
    return sg.MultiDRLEngine(engines)


def multi_result(multi, res):
    """Histories, final masters, adversary masters and sigmas of every population."""
    out = {}
    for k, (pol, hist) in enumerate(res):
        e = multi.engines[k]
        out[f"w{k}"] = pol.get_weights().numpy()
        out[f"sigma{k}"] = np.float64(e.mm_evolver.sigma)
        if e.use_arl:
            out[f"adv{k}"] = e.adv_evolver.master_policy.get_weights().numpy()
            out[f"asigma{k}"] = np.float64(e.adv_evolver.sigma)
        for key, v in hist.items():
            out[f"h{k}_{key}"] = np.array(v, np.float64)
    return out


def multi_train_rank(rank, world, port, P, gens, outdir, val_mode, arl, table_path=""):
    """MultiDRLEngine (3 populations, two assets) over `world` ranks sharing one
    GPU: every population's shard rolled out per rank, one gloo all-gather of
    the K records, then the multi-population tell/validation (best) or GA
    step (fused) on the gathered records -- the cross-rank record addressing
    (i / n) * K * record + k * stride + (i % n) * size with i / n > 0."""
    dist = _setup(rank, world, port)
    try:
        import sgmm_pkg
        sg = sgmm_pkg.load()
        if table_path:
            from sgmm_amd import _lib
            _lib.plan_set(policy_path=table_path)
        tr, va, st = multi_workload()
        multi = multi_engines(sg, P, arl, os.path.join(outdir, f"ck{rank}"), val_mode)
        sess = multi.session(tr, va, st, generations=gens)
        assert sess.world == world and sess.sharded and sess.best_val == (val_mode == "best")
        res = multi.train(tr, va, st, generations=gens)
        np.savez(os.path.join(outdir, f"m{rank}.npz"), **multi_result(multi, res))
    finally:
        dist.destroy_process_group()


def train_rank(rank, world, port, P, gens, outdir, backend="gloo"):
    """DRLEngine over `world` ranks sharing one GPU (gloo exchange staged
    through host memory): saves the history and the final master."""
    dist = _setup(rank, world, port, backend)
    try:
        import torch
        sg, tr, va, st, _ = workload(P, T=400, Tv=150)
        torch.manual_seed(0)
        eng = sg.DRLEngine(pop_size=P, phi=0.0005, tick_size=0.001, save_dir=os.path.join(outdir, f"ck{rank}"),
                           hidden_dim=16, rng="device", seed=11, verbose=False, sync_every=4, patience=3)
        pol, hist = eng.train(tr, va, st, generations=gens)
        np.savez(os.path.join(outdir, f"t{rank}.npz"), w=pol.get_weights().numpy(),
                 sigma=eng.mm_evolver.sigma, **{k: np.array(v, np.float64) for k, v in hist.items()})
    finally:
        dist.destroy_process_group()
