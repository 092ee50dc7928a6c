"""Microbenchmark: the latency of a LONE frontier walk with one, two or four waves
per walk (lane split), on GA-trained populations -- what a heavy walk at the end of
config 3's launch (alone on its SIMD) would gain from being finished with more waves.
Trains config 3 (bench.make_engine) for G generations, materializes generation G's
population, and times k_policy_frontier over n episodes of each population
(n << SIMDs: every walk alone on its SIMD) with groups=1 and lane_split 1 / 2 / 4.
    python tools/mb_ls_latency.py [G=15] [n=64]"""
import os
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import numpy as np
import torch

import bench
import sgmm_pkg

sg = sgmm_pkg.load()
from sgmm_amd import _lib
from sgmm_amd.model import genome_size

G_TRAIN = int(sys.argv[1]) if len(sys.argv) > 1 else 15
N = int(sys.argv[2]) if len(sys.argv) > 2 else 64
DEV = torch.device("cuda")
spec = dict(bench.CONFIGS[3])
P, H, T, K = spec["P"], spec["H"], spec["T"], len(spec["pops"])
Gs = genome_size(H)
data = bench.bundles(spec)
tr = [data[a][0] for _, _, a in spec["pops"]]
va = [data[a][1] for _, _, a in spec["pops"]]
st = [data[a][2] for _, _, a in spec["pops"]]
L = _lib.load()
eng = bench.make_engine(sg, spec, P, tempfile.mkdtemp(), None, True, "auto")
sess = eng.session(tr, va, st, generations=G_TRAIN + 1)
sess.steps(0, G_TRAIN)
torch.cuda.synchronize()
pop = torch.empty((K * P, Gs), dtype=torch.float32, device=DEV)
for k, e in enumerate(eng.engines):
    _lib.check(L.sgmm_ga_ask(_lib.ptr(sess.masters[k]), Gs, _lib.ptr(sess.states[k]), 0, e.seed, 0, P,
                             _lib.ptr(pop[k * P:]), Gs, _lib.stream_ptr()), "sgmm_ga_ask")
ticks = sg.TickStore()
seg = ticks.segments[ticks.add(tr[0], st[0])]
ticks.to(DEV)
params = sg.params_tensor([sg.EnvConfig(phi=phi, tick_size=tick) for phi, tick, _ in spec["pops"]], DEV)
roll = sg.RolloutEngine(DEV)
print(f"config 3 trained {G_TRAIN} generations; {N} episodes per launch (one walk per SIMD at most)")
for k in range(K):
    idx = np.arange(k * P, k * P + N)
    eps = sg.EpisodeBatch(idx, np.full(N, seg[0]), np.full(N, T), np.full(N, k)).to(DEV)
    res, ref = {}, None
    for ls in (1, 2, 4):
        with _lib.plan(policy_path="frontier", groups=1, lane_split=ls, min_eps=1):
            roll.fitness(ticks, eps, params, pop, H)
            _lib.profile_read()
            _lib.profile_enable(True)
            for _ in range(5):
                f, t = roll.fitness(ticks, eps, params, pop, H)
            kt = _lib.profile_read()
            _lib.profile_enable(False)
        out = (f.cpu().numpy(), t.cpu().numpy())
        ref = ref or out
        assert np.array_equal(ref[0], out[0]) and np.array_equal(ref[1], out[1])
        res[ls] = kt["policy_frontier"][0] / kt["policy_frontier"][1] * 1e3
    print(f"  population {k}: frontier kernel (the slowest of {N} lone walks) LS=1 {res[1]:.1f} us, "
          f"LS=2 {res[2]:.1f} us ({res[1] / res[2]:.2f}x), LS=4 {res[4]:.1f} us ({res[1] / res[4]:.2f}x)")
