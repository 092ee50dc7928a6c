"""Multi-rank path on CPU (gloo, world_size 2 and 3): population shards, the
per-rank fitness records and their one all-gather per generation, decoded
with the same addressing sgmm_ga_step uses (shard_n, shard_stride)."""
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import _shard_ranks as R


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_bounds_cover_population():
    import sgmm_pkg
    sgmm_pkg.load()
    from sgmm_amd.shard import shard_bounds, shard_capacity
    for P in (1, 2, 7, 64, 65, 511):
        for W in (1, 2, 3, 4, 8):
            n = shard_capacity(P, W)
            spans = [shard_bounds(P, r, W) for r in range(W)]
            assert spans[0][0] == 0 and spans[-1][1] == P
            for (a0, a1), (b0, b1) in zip(spans, spans[1:]):
                assert a1 == b0
            for r, (i0, i1) in enumerate(spans):
                assert 0 <= i1 - i0 <= n
                for i in range(i0, i1):  # the kernel's addressing: shard i // n, slot i % n
                    assert i // n == r and i % n == i - i0


@pytest.mark.parametrize("P,world", [(7, 2), (64, 2), (7, 3), (2, 3)])
def test_records_all_gather(tmp_path, P, world):
    mp.spawn(R.records_rank, args=(world, _port(), P, str(tmp_path)), nprocs=world, join=True)
    from sgmm_amd.shard import read_gathered
    _, tr, va, st, pop = R.workload(P)
    f, t = R.oracle_fitness(pop, tr, st, 16, range(P))
    vf, vt = R.oracle_fitness(pop, va, st, 16, range(P))
    outs = [np.load(tmp_path / f"r{r}.npz") for r in range(world)]
    g0 = outs[0]["gathered"]
    n = int(outs[0]["n"])
    for o in outs:  # every rank holds the same gathered records
        assert np.array_equal(o["gathered"], g0)
        assert np.array_equal(o["pf"], f) and np.array_equal(o["pt"], t)
        assert np.array_equal(o["pvf"], vf) and np.array_equal(o["pvt"], vt)
    for i in range(P):
        assert read_gathered(g0, i, n, "train_f") == f[i]
        assert read_gathered(g0, i, n, "train_t") == t[i]
        assert read_gathered(g0, i, n, "val_f") == vf[i]
        assert read_gathered(g0, i, n, "val_t") == vt[i]
    dec = np.array([read_gathered(g0, i, n, "train_f") for i in range(P)])
    assert int(np.argmax(dec)) == int(np.argmax(f))
