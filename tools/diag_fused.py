"""Fused vs separate path scan over a whole training session (diagnostic).

Trains config C for G generations twice with the same seeds -- the path scans
fused into the frontier launch, then the separate scan launch -- and compares
every population's history rows (best index, train fitness / trades,
validation) and final masters bit for bit; prints the first differences.

    python tools/diag_fused.py [config=3] [generations=30] [graph=1]
"""
import sys
import tempfile
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402
import sgmm_pkg  # noqa: E402


def run(fused, config, gens, graph):
    sgmm = sgmm_pkg.load()
    from sgmm_amd import _lib
    from sgmm_amd.drl_engine import HIST_DTYPE
    spec = dict(bench.CONFIGS[config])
    data = bench.bundles(spec)
    tr = [data[a][0] for _, _, a in spec["pops"]]
    va = [data[a][1] for _, _, a in spec["pops"]]
    st = [data[a][2] for _, _, a in spec["pops"]]
    with _lib.plan(fused_scan=fused):
        eng = bench.make_engine(sgmm, spec, spec["P"], tempfile.mkdtemp(), None, bool(graph), "auto")
        sess = eng.session(tr, va, st, generations=gens)
        sess.steps(0, gens)
        torch.cuda.synchronize()
        K = len(spec["pops"])
        rows = sess.hist[:, :gens].cpu().numpy().reshape(K, gens, -1).view(HIST_DTYPE).reshape(K, gens)
        masters = [m.cpu().numpy().copy() for m in sess.masters]
        sess.finish()
    return rows, masters


def main():
    config = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    gens = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    graph = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    a_rows, a_m = run(1, config, gens, graph)
    b_rows, b_m = run(0, config, gens, graph)
    bad = 0
    for k in range(a_rows.shape[0]):
        for g in range(gens):
            ra, rb = a_rows[k, g], b_rows[k, g]
            if ra.tobytes() != rb.tobytes():
                bad += 1
                if bad <= 12:
                    print(f"pop {k} gen {g}: fused {ra} separate {rb}")
    for k, (x, y) in enumerate(zip(a_m, b_m)):
        if x.tobytes() != y.tobytes():
            print(f"pop {k}: masters differ")
            bad += 1
    print("DIFFERENCES", bad, "of", a_rows.size, "history rows")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
