"""SGU2 inference against the reference's SGU2.predict on
its own checkpoints (tests/golden/g8_sgu2.npz, gen_golden_sgu2.py).

Tolerance: the reference evaluates the LSTM in float32 on the CPU (oneDNN /
BLAS summation order, libm transcendentals); the kernel in float32 on the GPU
(packed FMAs over even/odd columns, hardware exp2/rcp for sigmoid and tanh).
Both are compared with |out - want| <= ATOL + RTOL * |want| (ATOL = RTOL =
2e-6 on outputs of magnitude <= ~3; measured: reference vs float64 3.3e-7,
kernel vs reference 6.0e-7).  The scaler (float32 elementwise) is bit-exact."""
import numpy as np
import pytest
import torch

import sgu2_oracle as so
from conftest import has_gpu

ATOL = RTOL = 2e-6
gpu = pytest.mark.skipif(not has_gpu(), reason="needs a HIP device")


def close(a, want):
    a, want = np.asarray(a, np.float64).reshape(-1), np.asarray(want, np.float64).reshape(-1)
    return a.shape == want.shape and bool(np.all(np.abs(a - want) <= ATOL + RTOL * np.abs(want)))


@pytest.fixture(scope="module")
def g8(golden):
    return golden("g8_sgu2.npz")


def test_oracle_matches_reference(g8):
    xs = so.scale(g8["X"], g8["mean"], g8["std"])
    assert np.array_equal(xs, g8["X_scaled_f32"])
    for k in range(3):
        assert close(so.forward(g8[f"w{k}"], xs), g8[f"y{k}"]), k
        assert close(so.forward(g8[f"w{k}"], g8["X"]), g8[f"y{k}_raw"]), k


def test_scaler_and_checkpoint_layout(sgmm, g8):
    from sgmm_amd.gate_units import SGU2, StandardScaler3D
    sc = StandardScaler3D()
    sc.fit(g8["X"])
    assert sc.mean.dtype == np.float32 and np.array_equal(sc.mean.reshape(-1), g8["mean"])
    assert np.array_equal(sc.std.reshape(-1), g8["std"])
    assert np.array_equal(sc.transform(g8["X"]), g8["X_scaled_f32"])
    m = SGU2(input_size=1, hidden_size=10)
    w = g8["w0"]
    parts = so.unpack(w)
    sd = {k: torch.from_numpy(np.asarray(p, np.float32)) for k, p in zip(
        ("lstm.weight_ih_l0", "lstm.weight_hh_l0", "lstm.bias_ih_l0", "lstm.bias_hh_l0", "fc.weight", "fc.bias"), parts)}
    m.model.load_state_dict(sd)
    assert np.array_equal(m.model.flat_weights().numpy(), w)


def test_argument_errors_need_no_gpu(sgmm):
    import ctypes
    from sgmm_amd import _lib
    L = _lib.load()
    p = ctypes.c_void_p(8)
    assert L.sgmm_sgu2_forward(p, 12, p, 4, 10, None, None, p, None) == -1
    assert b"hidden" in L.sgmm_last_error()
    assert L.sgmm_sgu2_forward(p, 10, p, 4, 10, p, None, p, None) == -1
    assert L.sgmm_sgu2_forward(None, 10, p, 4, 10, None, None, p, None) == -1


def _model(g8, k):
    from sgmm_amd.gate_units import SGU2
    m = SGU2(1, 10)
    sd = {n: torch.from_numpy(np.asarray(p, np.float32)) for n, p in zip(
        ("lstm.weight_ih_l0", "lstm.weight_hh_l0", "lstm.bias_ih_l0", "lstm.bias_hh_l0", "fc.weight", "fc.bias"),
        so.unpack(g8[f"w{k}"]))}
    m.model.load_state_dict(sd)
    return m


@pytest.mark.gpu
@gpu
def test_predict_matches_reference(sgmm, g8):
    from sgmm_amd.gate_units import StandardScaler3D
    sc = StandardScaler3D()
    sc.fit(g8["X"])
    for k in range(3):
        m = _model(g8, k)
        assert close(m.predict(g8["X"]), g8[f"y{k}_raw"]), k
        assert close(m.predict(g8["X_scaled_f32"]), g8[f"y{k}"]), k
        X = torch.from_numpy(g8["X"]).cuda()
        assert close(m.predict_device(X, sc).cpu().numpy(), g8[f"y{k}"]), k   # scaler in the kernel
        assert m.predict(g8["X"]).shape == (len(g8["X"]), 1)


@pytest.mark.gpu
@gpu
def test_predict_many_windows_matches_oracle(sgmm, g8):
    rng = np.random.default_rng(3)
    X = (rng.standard_t(4, size=(200_003, 10, 1)) * 3e-4).astype(np.float32)
    X[::7] = 0.0
    for k in (0, 1):
        m = _model(g8, k)
        got = m.predict_device(torch.from_numpy(X).cuda()).cpu().numpy()
        assert close(got, so.forward(g8[f"w{k}"], X)), k
    empty = _model(g8, 0).predict_device(torch.zeros((0, 10), dtype=torch.float32, device="cuda"))
    assert empty.numel() == 0


@pytest.mark.gpu
@gpu
def test_bundle_with_device_sgu2(sgmm, golden, tmp_path):
    """load_signals_bundle with this package's SGU2 + a float32 scaler runs SGU2
    on the device windows of all days in one launch; equal to the host path
    (the same kernel fed the host windows) and within tolerance of the oracle."""
    import pandas as pd
    from sgmm_amd.bundle import load_signals_bundle
    from sgmm_amd.gate_units import StandardScaler3D
    g6, g8 = golden("g6_bundle.npz"), golden("g8_sgu2.npz")
    dates = [str(d) for d in g6["dates"]]
    for k, d in enumerate(dates):
        for kind in ("snap", "tick"):
            p = tmp_path / "data" / "SYN" / kind
            p.mkdir(parents=True, exist_ok=True)
            pd.DataFrame({c[len(f"d{k}_{kind}_"):]: g6[c] for c in g6 if c.startswith(f"d{k}_{kind}_")}) \
                .to_parquet(p / f"{d}.parquet")
    sc = StandardScaler3D()
    sc.fit(np.concatenate([g6[f"d{k}_sgu2_X"] for k in range(len(dates)) if g6[f"d{k}_sgu2_X"].ndim == 3]))
    m2 = _model(g8, 0)

    class HostM2:  # any non-package model: the reference's host path
        def predict(self, X):
            return m2.predict(X)

    class M1:
        def predict(self, X):
            return np.asarray(X.iloc[:, 0].values, dtype=np.float32)

    def feats():
        it = iter([g6[f"d{k}_sgu1_f0"] for k in range(len(dates))])
        return lambda bars: (lambda v: pd.DataFrame({"f0": v, "label": np.zeros(len(v))}))(next(it))

    fused = load_signals_bundle("SYN", dates, M1(), m2, sc, sgu1_features=feats(), data_root=str(tmp_path))
    host = load_signals_bundle("SYN", dates, M1(), HostM2(), sc, sgu1_features=feats(), data_root=str(tmp_path))
    for a, b in zip(fused, host):
        assert np.array_equal(a, b, equal_nan=True)
    assert fused[1].dtype == np.float32
    # s2 against the oracle on the reference's windows (aligned tails, last step dropped)
    want = []
    for k in range(len(dates)):
        X = g6[f"d{k}_sgu2_X"]
        if X.ndim != 3:
            continue
        y = so.forward(g8["w0"], so.scale(X, sc.mean, sc.std)).reshape(-1)
        n = min(len(g6[f"d{k}_sgu1_f0"]), len(y))
        want.append(y[-n:][:-1])
    assert close(fused[1], np.concatenate(want))
