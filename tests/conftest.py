import os
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
GOLDEN = ROOT / "tests" / "golden"
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


@pytest.fixture(scope="session")
def golden():
    def load(name):
        return dict(np.load(GOLDEN / name, allow_pickle=False))
    return load


@pytest.fixture(scope="session")
def sgmm():
    import sgmm_pkg
    return sgmm_pkg.load()


@pytest.fixture(scope="session")
def oracle():
    import oracle as orc
    return orc


def episodes_from_fixture(d):
    """Yield per-episode dicts from a g2/g3 style stacked fixture."""
    for e in range(len(d["ep_off"])):
        o, n = int(d["ep_off"][e]), int(d["ep_len"][e])
        sl = slice(o, o + n)
        H = int(d["H"][e])
        G = H * H + 7 * H + 2
        yield dict(
            e=e, H=H, mm=d["mm"][e][:G], adv=d["adv"][e] if d["arl"][e] else None,
            s1=d["s1"][sl], s2=d["s2"][sl], s1n=d["s1n"][sl], s2n=d["s2n"][sl],
            mid=d["mid"][sl], ask=d["ask"][sl], bid=d["bid"][sl],
            buy_max=d["buy_max"][sl], sell_min=d["sell_min"][sl],
            phi=float(d["phi"][e]), tick=float(d["tick"][e]), fee=float(d["fee"][e]),
            fitness=float(d["fitness"][e]), trades=int(d["trades"][e]),
            tie_margin=float(d["tie_margin"][e]), raw=d["raw"][sl],
            stats=d["stats"][e], stats_nb=bool(d["stats_nb"][e]),
            tr={k[3:]: d[k][sl] for k in d if k.startswith("tr_")},
        )


def stats_dict(st, nb):
    """Rebuild train_stats with the scalar types the reference saw."""
    if nb:
        return {"s1_m": np.float32(st[0]), "s1_s": np.float64(st[1]),
                "s2_m": np.float32(st[2]), "s2_s": np.float64(st[3])}
    return {"s1_m": np.float32(st[0]), "s1_s": np.float32(st[1]),
            "s2_m": np.float32(st[2]), "s2_s": np.float32(st[3])}


def has_gpu():
    if os.environ.get("SGMM_FORCE_NO_GPU"):
        return False
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def near_tie(raw, scale=5.0, ulps=64):
    """True where raw*scale lies within `ulps` float32 ulps (relative to its
    magnitude) of a rounding boundary k+1/2 -- where an fp32 summation-order
    difference may legitimately flip the rounded action."""
    v = raw.astype(np.float32) * np.float32(scale)
    dist = np.abs(v.astype(np.float64) - np.floor(v.astype(np.float64)) - 0.5)
    return dist <= ulps * np.spacing(np.abs(v)).astype(np.float64) + 1e-7


def agree_until_justified_divergence(act_ours, act_ref, raw_ref, scale=5.0):
    """Index up to which two action streams must agree.

    Returns len if identical; otherwise the first differing step, which must be
    a near-tie step of the reference's raw output (else AssertionError)."""
    diff = np.nonzero(np.any(act_ours != act_ref, axis=1))[0]
    if len(diff) == 0:
        return len(act_ours)
    t = int(diff[0])
    assert np.any(near_tie(raw_ref[t], scale)), (t, act_ours[t], act_ref[t], raw_ref[t])
    return t


@pytest.fixture
def plan(sgmm):
    """Launch-plan overrides for one test (sgmm_plan_set: policy_path, groups,
    lane_split, table_sp, spill, ...), restored to the default rules afterwards."""
    from sgmm_amd import _lib
    saved = {}

    def set_(**knobs):
        for k, v in _lib.plan_set(**knobs).items():
            saved.setdefault(k, v)

    yield set_
    _lib.plan_set(**saved)
