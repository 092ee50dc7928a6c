"""Debug: compare graph-replayed and eager generations buffer by buffer."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import numpy as np
import torch
import sgmm_pkg
sg = sgmm_pkg.load()
from sgmm_amd import synthetic

tr = synthetic.bundle_510300(600, seed=0)
va = synthetic.bundle_510300(150, seed=1)
st = synthetic.train_stats(tr)
snaps = {}
for use_graph in (False, True):
    eng = sg.DRLEngine(pop_size=24, phi=0.0005, tick_size=0.001, save_dir="/tmp/dbg", hidden_dim=16,
                       seed=42, val_mode="fused", use_graph=use_graph, verbose=False)
    s = eng.session(tr, va, st, generations=3)
    m0 = s.master.clone()
    s.step(0)
    torch.cuda.synchronize()
    snaps[use_graph] = dict(m0=m0.cpu(), pop=s.pop.cpu(), out0=s.out[0].cpu(), out1=s.out[1].cpu(),
                            master=s.master.cpu(), state=s.state.cpu(), hist=s.hist.cpu())
a, b = snaps[False], snaps[True]
for k in a:
    eq = torch.equal(a[k], b[k])
    print(k, "equal" if eq else "DIFF", "" if eq else (a[k].flatten()[:6], b[k].flatten()[:6]))
