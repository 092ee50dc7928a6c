"""Diagnostic: the validation launch's shape (K episodes of T ticks, H=32) on the
table paths -- the one-state-per-wave MFMA table (default for small launches),
v3 (MFMA, one wave per 64-tick chunk, the five states in turn) and the VALU table (one wave per (chunk, state)) -- kernel times by HIP events.
    python tools/mb_val_table.py [K=5] [T=912]"""
import os
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import numpy as np
import torch
import sgmm_pkg
sg = sgmm_pkg.load()
from sgmm_amd import _lib, synthetic
K = int(sys.argv[1]) if len(sys.argv) > 1 else 5
T = int(sys.argv[2]) if len(sys.argv) > 2 else 912
H = 32
dev = torch.device("cuda")
b = synthetic.bundle_510300(T, seed=3)
st = synthetic.train_stats(b)
ticks = sg.TickStore(); ticks.add(b, st); ticks.to(dev)
params = sg.params_tensor([sg.EnvConfig(phi=1e-4, tick_size=0.001)], dev)
pop = synthetic.population(K, H, sigma=0.1, seed=4).to(dev)
eb = sg.EpisodeBatch(np.arange(K), np.zeros(K), np.full(K, T), np.zeros(K)).to(dev)
out = {}
for path in ("table", "v3", "valu"):
    os.environ["SGMM_TABLE_PATH"] = "table" if path == "v3" else path
    os.environ["SGMM_TABLE_SP"] = "0" if path == "v3" else "1"
    eng = sg.RolloutEngine(dev)
    for _ in range(5):
        f, t = eng.fitness(ticks, eb, params, pop, H)
    torch.cuda.synchronize()
    _lib.profile_read()
    _lib.profile_enable(True)
    for _ in range(50):
        f, t = eng.fitness(ticks, eb, params, pop, H)
    torch.cuda.synchronize()
    prof = _lib.profile_read()
    _lib.profile_enable(False)
    out[path] = (f.cpu().numpy(), t.cpu().numpy())
    print(path, {k: round(v[0] * 1e3 / v[1], 2) for k, v in prof.items()}, "us per launch")
for k in ("v3", "valu"):
    assert np.array_equal(out["table"][0], out[k][0]) and np.array_equal(out["table"][1], out[k][1])
print("fitness identical")
