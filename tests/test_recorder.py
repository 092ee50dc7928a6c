"""Batched backtest recorder against the reference's
recorder frames (tests/golden/g7_recorder.npz, gen_golden_recorder.py):
CPU tests of the frame assembly, GPU tests of the traced backtests."""
import numpy as np
import pytest
import torch

from conftest import has_gpu

CASES = ("main_0", "main_1", "main_2")
gpu = [pytest.mark.gpu, pytest.mark.skipif(not has_gpu(), reason="needs a HIP device")]


@pytest.fixture(scope="module")
def g7(golden):
    return golden("g7_recorder.npz")


def bundle(g7):
    return tuple(g7[f"bundle_{k}"] for k in ("s1", "s2", "mid", "ask", "bid", "buy_max", "sell_min"))


def stats(g7):
    s = g7["stats"]  # the notebook's train_stats: float32 means, float64 stds
    return {"s1_m": np.float32(s[0]), "s1_s": np.float64(s[1]), "s2_m": np.float32(s[2]), "s2_s": np.float64(s[3])}


def assert_frame(df, g7, tag, dtypes=True):
    cols = [str(c) for c in g7[f"{tag}__columns"]]
    assert list(df.columns) == cols
    for c, dt in zip(cols, g7[f"{tag}__dtypes"]):
        v = df[c].to_numpy()
        if v.dtype == object:
            v = np.stack([np.asarray(x) for x in v])
        want = g7[f"{tag}__{c}"]
        assert v.shape == want.shape and np.array_equal(v.astype(np.float64), want.astype(np.float64),
                                                        equal_nan=True), (tag, c)
        if dtypes:
            assert str(df[c].dtype) == str(dt), (tag, c, df[c].dtype, dt)
            if c == "action":
                assert np.asarray(df[c].iloc[0]).dtype == want.dtype


@pytest.mark.parametrize("tag,schema", [("main_0", "backtest"), ("main_1", "backtest"), ("blind", "blind")])
def test_frame_assembly_matches_reference_recorder(sgmm, g7, tag, schema):
    """Device trace columns -> StrategyRecorder.to_dataframe, fed here with the
    reference's own per-step values (no GPU)."""
    from sgmm_amd.recorder import _frame
    cols = {"off_a": g7[f"{tag}__off_a"], "off_b": g7[f"{tag}__off_b"], "inventory": g7[f"{tag}__inventory"],
            "cash": g7[f"{tag}__cash"], "reward": g7[f"{tag}__reward"], "pnl": g7[f"{tag}__pnl_reward"],
            "fee_paid": g7[f"{tag}__fee_paid"]}
    if schema == "backtest":
        cols["fill_buy"], cols["fill_sell"] = g7[f"{tag}__fill_buy"], g7[f"{tag}__fill_sell"]
    else:  # the fixture keeps is_trade only; fills from the matching main run are not needed
        cols["fill_buy"] = g7[f"{tag}__is_trade"]
        cols["fill_sell"] = np.zeros_like(cols["fill_buy"])
    phi = float(g7[f"{tag}__phi_fee"][0])
    assert_frame(_frame(schema, cols, bundle(g7), phi), g7, tag)


def test_restated_loop_reproduces_reference_parquet(g7):
    """The fixture's main.py loop equals output/510300/arl/backtest_0.0001.parquet
    (values; that parquet's int32 columns come from its authors' platform)."""
    for c in g7["arl_parquet__columns"]:
        assert np.array_equal(g7[f"arl_parquet__{c}"].astype(np.float64), g7[f"main_0__{c}"].astype(np.float64)), c


@pytest.mark.parametrize("schema", ["backtest", "blind"])
def test_unknown_schema_and_empty_batch(sgmm, schema):
    from sgmm_amd.recorder import run_backtests
    assert run_backtests([], None, {}, 0.0, schema=schema) == []
    with pytest.raises(ValueError):
        run_backtests([], None, {}, 0.0, schema="detailed")


@pytest.mark.gpu
@pytest.mark.skipif(not has_gpu(), reason="needs a HIP device")
def test_backtests_one_launch_match_reference(sgmm, g7):
    """Three phi/fee backtests of the ARL checkpoint in one trace launch."""
    from sgmm_amd.recorder import run_backtests
    phis = [float(g7[f"{t}__phi_fee"][0]) for t in CASES]
    fees = [float(g7[f"{t}__phi_fee"][1]) for t in CASES]
    dfs = run_backtests([g7["genome"]] * 3, bundle(g7), stats(g7), phis, fees, 0.001)
    for df, tag in zip(dfs, CASES):
        assert_frame(df, g7, tag)
    assert_frame(dfs[0], g7, "arl_parquet", dtypes=False)


@pytest.mark.gpu
@pytest.mark.skipif(not has_gpu(), reason="needs a HIP device")
def test_blind_test_matches_reference(sgmm, g7):
    from sgmm_amd.model import TradingPolicy
    from sgmm_amd.recorder import blind_test
    pol = TradingPolicy()
    pol.set_weights(torch.from_numpy(g7["genome"]))
    phi, fee = (float(x) for x in g7["blind__phi_fee"])
    assert_frame(blind_test(pol, bundle(g7), stats(g7), phi, 0.001, fee), g7, "blind")


@pytest.mark.gpu
@pytest.mark.skipif(not has_gpu(), reason="needs a HIP device")
def test_run_drl_backtest_writes_reference_parquet(sgmm, g7, tmp_path, monkeypatch):
    import pandas as pd
    from sgmm_amd.model import genome_to_state_dict
    from sgmm_amd.recorder import run_drl_backtest
    w = tmp_path / "agent.pth"
    torch.save(genome_to_state_dict(g7["genome"], 32), w)
    monkeypatch.chdir(tmp_path)
    assert run_drl_backtest("510300", "arl", str(tmp_path / "missing.pth"), bundle(g7), 0.0001, 0.0, stats(g7)) is None
    df = run_drl_backtest("510300", "arl", str(w), bundle(g7), 0.0001, 0.0, stats(g7))
    back = pd.read_parquet(tmp_path / "output/510300/arl/backtest_0.0001.parquet")
    assert_frame(back, g7, "main_0")
    assert_frame(df, g7, "main_0")
