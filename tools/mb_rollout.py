"""Microbenchmark: per-kernel time of sgmm_rollout_fitness vs population size."""
import json
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import numpy as np
import torch
import sgmm_pkg
sg = sgmm_pkg.load()
from sgmm_amd import _lib, synthetic

T = int(sys.argv[1]) if len(sys.argv) > 1 else 3600
H = int(sys.argv[2]) if len(sys.argv) > 2 else 16
dev = torch.device("cuda")
b = synthetic.bundle_510300(T, seed=0)
st = synthetic.train_stats(b)
ticks = sg.TickStore(); ticks.add(b, st); ticks.to(dev)
params = sg.params_tensor([sg.EnvConfig(phi=1e-4, tick_size=0.001)], dev)
eng = sg.RolloutEngine(dev)
res = {}
PS = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else (1, 16, 64, 256, 1024, 4096)
for P in PS:
    pop = synthetic.population(P, H, sigma=0.05, seed=1).to(dev)
    eps = sg.EpisodeBatch(np.arange(P), np.zeros(P), np.full(P, T), np.zeros(P)).to(dev)
    out = eng.fitness(ticks, eps, params, pop, H)
    torch.cuda.synchronize()
    _lib.profile_read()
    _lib.profile_enable(True)
    n = 10
    for _ in range(n):
        eng.fitness(ticks, eps, params, pop, H, out=out)
    torch.cuda.synchronize()
    _lib.profile_enable(False)
    pr = _lib.profile_read()
    res[P] = {k: round(1e3 * v[0] / v[1], 1) for k, v in pr.items()}
    tab = pr["policy_table"][0] / n * 1e-3
    res[P]["table_TFLOPs_alg"] = round(P * T * 2 * (5 * H + H * H) / tab / 1e12, 2)
    res[P]["Gsteps_per_s_kernels"] = round(P * T / ((pr["policy_table"][0] + pr["path_scan"][0]) / n * 1e-3) / 1e9, 2)
print(json.dumps(res, indent=1))
