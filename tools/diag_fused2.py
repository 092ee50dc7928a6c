"""The trained-state test's flow (tests/test_gpu_trained_state.py::_pin_trained),
with the generation-`gens` history rows printed: train config 3 `gens`
generations, optionally run a standalone fitness launch (step 1), then one more
session generation; prints each population's row and the session state.

    python tools/diag_fused2.py [gens=24] [standalone=1] [fused=1]
"""
import os
import sys
import tempfile
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402
import sgmm_pkg  # noqa: E402


def main():
    gens = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    standalone = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    fused = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    sgmm = sgmm_pkg.load()
    from sgmm_amd import _lib
    from sgmm_amd.drl_engine import HIST_DTYPE
    from sgmm_amd.model import genome_size
    _lib.plan_set(fused_scan=fused)
    spec = dict(bench.CONFIGS[3])
    P, H, T = spec["P"], spec["H"], spec["T"]
    K = len(spec["pops"])
    G = genome_size(H)
    data = bench.bundles(spec)
    tr = [data[a][0] for _, _, a in spec["pops"]]
    va = [data[a][1] for _, _, a in spec["pops"]]
    st = [data[a][2] for _, _, a in spec["pops"]]
    eng = bench.make_engine(sgmm, spec, P, tempfile.mkdtemp(), None, os.environ.get("DIAG_GRAPH", "1") == "1", "auto")
    sess = eng.session(tr, va, st, generations=gens + 1)
    sess.steps(0, gens)
    torch.cuda.synchronize()
    L, s = sess.L, _lib.stream_ptr()
    pop = torch.empty((K * P, G), dtype=torch.float32, device="cuda")
    for k, e in enumerate(eng.engines):
        _lib.check(L.sgmm_ga_ask(_lib.ptr(sess.masters[k]), G, _lib.ptr(sess.states[k]), 0, e.seed, 0, P,
                                 _lib.ptr(pop[k * P:]), G, s), "sgmm_ga_ask")
    got = None
    if standalone:
        ticks = sgmm.TickStore()
        seg = {}
        for k in range(K):
            if id(tr[k]) not in seg:
                seg[id(tr[k])] = ticks.segments[ticks.add(tr[k], st[k])]
        ticks.to("cuda")
        offs = np.concatenate([np.full(P, seg[id(tr[k])][0]) for k in range(K)])
        eps = sgmm.EpisodeBatch(np.arange(K * P), offs, np.full(K * P, T), np.repeat(np.arange(K), P)).to("cuda")
        params = sgmm.params_tensor([sgmm.EnvConfig(phi=phi, tick_size=tick) for phi, tick, _ in spec["pops"]], "cuda")
        r2 = sgmm.RolloutEngine("cuda")
        sa = {}
        if "DIAG_SA_FUSED" in os.environ:
            sa["fused_scan"] = int(os.environ["DIAG_SA_FUSED"])
        if "DIAG_SA_GROUPS" in os.environ:
            sa["groups"] = int(os.environ["DIAG_SA_GROUPS"])
        with _lib.plan(**sa):
            fit, trd = r2.fitness(ticks, eps, params, pop, H, None)
        torch.cuda.synchronize()
        print("standalone ws", hex(r2._ws.data_ptr()), r2._ws.numel())
        del r2
        got = fit.cpu().numpy().reshape(K, P)
    print("states before:", [bytes(x.cpu().numpy().tobytes()[:64]).hex() for x in sess.states][:1])
    a256 = lambda x: (x + 255) & ~255
    n, steps = K * P, K * P * T
    nc, nfr = steps // 64 + n + 1, n * 64 * 2
    off = a256(max(nc, nfr) * 8) + a256(max(nc * 8, nfr * 32)) + a256(nfr * 4) + 2 * a256(n * 64 * 4)
    ws = sess.roll._ws
    arr = lambda: ws[off:off + 4 * n].cpu().numpy().view(np.uint32)
    print("session ws", hex(ws.data_ptr()), ws.numel(), "arrive nonzero before:", int((arr() != 0).sum()))
    sess.steps(gens, 1)
    torch.cuda.synchronize()
    a = arr()
    print("arrive nonzero after:", int((a != 0).sum()), "values", np.unique(a)[:10])
    f24 = sess.rec.f[:n].cpu().numpy()
    order = sess.walk_order.cpu().numpy()
    print("walk order is a permutation:", bool(np.array_equal(np.sort(order), np.arange(n))))
    if got is not None:
        bad = np.nonzero(f24 != got.reshape(-1))[0]
        print("episodes whose gen-24 record differs from the standalone:", len(bad), bad[:20])
        pos = np.argsort(order)  # position of each episode in the walk order
        print("their order positions:", pos[bad][:20], "counters:", a[bad][:20])
        nz = np.nonzero(a)[0]
        print("nonzero-counter episodes:", nz[:20], "positions", pos[nz][:20], "values", a[nz][:20])
    rows = sess.hist[:, gens].cpu().numpy().reshape(K, -1).view(HIST_DTYPE).reshape(K)
    prev = sess.hist[:, gens - 1].cpu().numpy().reshape(K, -1).view(HIST_DTYPE).reshape(K)
    for k in range(K):
        extra = "" if got is None else f" argmax(standalone)={int(np.argmax(got[k]))} max={got[k].max()!r}"
        print(f"pop {k}: gen {gens} row {rows[k]} | gen {gens - 1} row {prev[k]}{extra}")
    print("states after:", [x.cpu().numpy().tobytes()[:64].hex() for x in sess.states][:1])
    sess.finish()


if __name__ == "__main__":
    main()
