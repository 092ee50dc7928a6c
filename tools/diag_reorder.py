import sys, tempfile
sys.path.insert(0, "/root/repo")
import numpy as np, torch, bench, sgmm_pkg
sg = sgmm_pkg.load()
spec = dict(bench.CONFIGS[3]); P = spec["P"]
data = bench.bundles(spec)
tr = [data[a][0] for _, _, a in spec["pops"]]; va = [data[a][1] for _, _, a in spec["pops"]]; st = [data[a][2] for _, _, a in spec["pops"]]
eng = bench.make_engine(sg, spec, P, tempfile.mkdtemp(), None, False, "auto")
sess = eng.session(tr, va, st, generations=12)
print("best_val", sess.best_val, "walk_order ptr", sess.pops.walk_order, sess.walk_order.data_ptr())
for g in range(10):
    sess.step(g); torch.cuda.synchronize()
    print(g, sess.walk_order.cpu().numpy()[::512], sess.eps.dev["order"].cpu().numpy()[::512])
