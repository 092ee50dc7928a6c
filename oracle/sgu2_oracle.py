"""TEST INFRASTRUCTURE ONLY -- CPU restatement of SGU2 inference (SURVEY §8f
row 4) used by tests/ as the checker of the HIP kernel; the product path never
imports it.

  scale     utils/scaler.py:9-18  StandardScaler3D: mean/std of float32 windows
            are float32 (np.mean / np.std keep the dtype, + 1e-9 too), so
            transform is (X - mean) / std in float32
  forward   models/GateUnits.py:42-54  nn.LSTM(1, H, batch_first) over the
            window (PyTorch gate order i, f, g, o; c = f*c + i*g,
            h = o*tanh(c)), last step -> Dropout (identity in eval) -> Linear(H, 1)

Evaluated in float64 from the float32 weights and inputs: the reference's
float32 CPU LSTM (oneDNN / BLAS summation order unpinned) lies within
tests' stated tolerance of it.  Pinned by tests/golden/g8_sgu2.npz (the
reference's SGU2.predict on its own checkpoints, gen_golden_sgu2.py).
"""
from __future__ import annotations

import numpy as np


def unpack(w: np.ndarray, hidden: int = 10, input_size: int = 1):
    """Flat float32 weights in state_dict order (weight_ih, weight_hh, bias_ih,
    bias_hh, fc.weight, fc.bias) -> arrays."""
    H, I = hidden, input_size
    sizes = (4 * H * I, 4 * H * H, 4 * H, 4 * H, H, 1)
    parts, o = [], 0
    for n in sizes:
        parts.append(np.asarray(w[o:o + n], np.float64))
        o += n
    assert o == len(w), (o, len(w))
    return (parts[0].reshape(4 * H, I), parts[1].reshape(4 * H, H), parts[2], parts[3],
            parts[4].reshape(1, H), parts[5])


def scale(X, mean, std) -> np.ndarray:
    """StandardScaler3D.transform of float32 windows with a float32 fit."""
    X = np.asarray(X, np.float32)
    return (X - np.asarray(mean, np.float32)) / np.asarray(std, np.float32)


def forward(w, X, hidden: int = 10) -> np.ndarray:
    """SGU2Model.forward in eval mode: X [n, T, I] -> [n, 1]."""
    w_ih, w_hh, b_ih, b_hh, fc_w, fc_b = unpack(w, hidden, np.asarray(X).shape[2])
    X = np.asarray(X, np.float64)
    n, T, _ = X.shape
    H = hidden
    h = np.zeros((n, H))
    c = np.zeros((n, H))
    sig = lambda v: 1.0 / (1.0 + np.exp(-v))
    for t in range(T):
        g = X[:, t, :] @ w_ih.T + b_ih + h @ w_hh.T + b_hh
        i, f, gg, o = sig(g[:, :H]), sig(g[:, H:2 * H]), np.tanh(g[:, 2 * H:3 * H]), sig(g[:, 3 * H:])
        c = f * c + i * gg
        h = o * np.tanh(c)
    return h @ fc_w.T + fc_b
