"""Experiment: config 3's five populations as S independent sessions on S HIP
streams (each population's generations are unchanged; only the launches of
different populations may overlap on the GPU), against one session.

    python tools/mb_streams.py --split 1 2 5 --steps 20 --warmup 5
"""
import argparse
import json
import os
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402


def groups_of(K, S):
    return [list(range(K))[i::S] for i in range(S)] if S > 1 else [list(range(K))]


def run(S, args, sgmm, spec, data):
    import torch
    K = len(spec["pops"])
    gs = groups_of(K, S)
    tmp = tempfile.mkdtemp(prefix="sgmm_streams_")
    sessions, streams = [], []
    for gi, g in enumerate(gs):
        sub = dict(spec)
        sub["pops"] = [spec["pops"][k] for k in g]
        eng = bench.make_engine(sgmm, sub, spec["P"], tmp, None, not args.no_graph, "best", seed0=1234 + 101 * gi)
        tr = [data[a][0] for _, _, a in sub["pops"]]
        va = [data[a][1] for _, _, a in sub["pops"]]
        st = [data[a][2] for _, _, a in sub["pops"]]
        sess = eng.session(tr, va, st, generations=args.warmup + args.steps)
        s = torch.cuda.Stream() if S > 1 else torch.cuda.current_stream()
        with torch.cuda.stream(s):
            sess.steps(0, args.warmup)
            sess.capture()
        sessions.append(sess)
        streams.append(s)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for sess, s in zip(sessions, streams):
        with torch.cuda.stream(s):
            sess.steps(args.warmup, args.steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    res = [r for sess in sessions for r in sess.finish()]
    value = K * spec["P"] * spec["T"] * args.steps / dt
    return {"S": S, "groups": gs, "ms_per_gen": dt / args.steps * 1e3, "G": value / 1e9,
            "final_train_f": [float(h["train_f"][-1]) for _, h in res]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--split", type=int, nargs="+", default=[1, 2, 5])
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--no-graph", action="store_true")
    args = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    import sgmm_pkg
    sgmm = sgmm_pkg.load()
    spec = dict(bench.CONFIGS[args.config])
    data = bench.bundles(spec)
    for r in range(args.reps):
        for S in args.split:
            print(json.dumps(run(S, args, sgmm, spec, data)), flush=True)


if __name__ == "__main__":
    main()
