"""The multi-GPU generation on RCCL (torch.distributed "nccl" = RCCL on ROCm),
on the one GPU a test box has: a world-size-1 nccl group, the sharded path
forced (DRLEngine(exchange="always"): asked rollout -> all_gather_into_tensor of
the fitness records -> GA step), and the all-gather captured INSIDE the
generation HIP graph -- one graph per generation and one per batch of
generations, the same replay a multi-rank run uses.  The result must equal the
unsharded one-process training bit for bit (histories, masters, sigma).
Reference: Env/drl_engine.py:91-125 (Pool.starmap over the population, tell).
"""
import os
import socket

import numpy as np
import pytest
import torch

from conftest import has_gpu

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not has_gpu(), reason="needs a HIP device")]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture
def nccl_world1():
    import torch.distributed as dist
    if not dist.is_nccl_available():
        pytest.skip("no nccl (RCCL) backend")
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    torch.cuda.set_device(0)
    for attempt in range(5):  # a probed free port can be taken before the store binds it
        try:
            dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                                    device_id=torch.device("cuda", 0))
            break
        except dist.DistNetworkError:
            if attempt == 4:
                raise
    try:
        yield dist
    finally:
        dist.destroy_process_group()


def _bundles():
    from sgmm_amd import synthetic
    tr = synthetic.bundle_510300(700, seed=61)
    va = synthetic.bundle_510300(160, seed=62)
    return tr, va, synthetic.train_stats(tr)


def _multi(sgmm, tmp, exchange, arl=False, val_mode="fused"):
    engines = []
    for k, phi in enumerate((0.0001, 0.005)):
        torch.manual_seed(300 + k)
        engines.append(sgmm.DRLEngine(pop_size=40, phi=phi, tick_size=0.001, use_arl=arl, save_dir=str(tmp),
                                      hidden_dim=16, rng="device", seed=77 + k, val_mode=val_mode, sync_every=8,
                                      patience=3, verbose=False, exchange=exchange))
    return sgmm.MultiDRLEngine(engines)


@pytest.mark.parametrize("arl,val_mode", [(False, "fused"), (True, "fused"), (False, "best"), (True, "best")],
                         ids=["mm", "arl", "mm-best", "arl-best"])
def test_rccl_exchange_in_graph_equals_single_process(sgmm, tmp_path, nccl_world1, arl, val_mode):
    """best: the ranks gather training records only, then every rank runs the
    tell (sgmm_ga_tell_multi) and validates the new masters
    (sgmm_validate_multi), all inside the captured graphs; the reference
    result is the one-process fused training."""
    tr, va, st = _bundles()
    gens = 20  # one 8-generation batch graph twice, then 4 single-generation replays
    ref = _multi(sgmm, tmp_path / "ref", "auto", arl).train(tr, va, st, generations=gens)
    m = _multi(sgmm, tmp_path / "rccl", "always", arl, val_mode)
    sess = m.session(tr, va, st, generations=gens)
    assert sess.sharded and sess.world == 1
    for g0 in range(0, gens, 8):
        n = min(8, gens - g0)
        sess.steps(g0, n)
        if n == 8:
            sess.flush(g0 + n)
    assert sess.full_graph, getattr(sess, "capture_error", "")  # all-gather inside the graph
    assert sess.batch_graph is not None
    got = sess.finish()
    for (pa, ha), (pb, hb) in zip(ref, got):
        for key in ha:
            assert np.array_equal(np.array(ha[key], np.float64), np.array(hb[key], np.float64), equal_nan=True), key
        assert np.array_equal(pa.get_weights().numpy(), pb.get_weights().numpy())


def test_rccl_single_population_session(sgmm, tmp_path, nccl_world1):
    """DRLEngine (one population) on the same forced-exchange path."""
    tr, va, st = _bundles()
    out = {}
    for ex, vm in (("auto", "fused"), ("always", "fused"), ("always", "best"), ("auto", "best")):
        torch.manual_seed(5)
        e = sgmm.DRLEngine(pop_size=48, phi=0.001, tick_size=0.001, save_dir=str(tmp_path / (ex + vm)),
                           hidden_dim=32, rng="device", seed=9, sync_every=8, verbose=False, exchange=ex,
                           val_mode=vm, patience=3)
        sess = e.session(tr, va, st, generations=16)
        sess.steps(0, 16)
        if ex == "always":
            assert sess.full_graph, getattr(sess, "capture_error", "")
        assert sess.best_step == (vm == "best")
        pol, hist = sess.finish()
        out[ex + vm] = (pol.get_weights().numpy(), hist, e.mm_evolver.sigma)
    wa, ha, sa = out["autofused"]
    for k2 in ("alwaysfused", "alwaysbest", "autobest"):
        wb, hb, sb = out[k2]
        for key in ha:
            assert np.array_equal(np.array(ha[key], np.float64), np.array(hb[key], np.float64), equal_nan=True), \
                (k2, key)
        assert np.array_equal(wa, wb) and sa == sb, k2
