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
