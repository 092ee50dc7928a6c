"""SGU2 (the LSTM signal gate unit) inference on the GPU,
API-compatible with models/GateUnits.py:42-136 and utils/scaler.py.

``SGU2Model`` is the weight container and checkpoint format (state_dict keys
lstm.* / fc.* as GateUnits.py:42-47); ``SGU2.predict`` runs libsgmm.so's
sgmm_sgu2_forward over all windows in one launch.  ``predict_device`` takes
the windows already on the device (sgmm_bar_windows' output) and applies the
StandardScaler3D fit in the kernel, so the bundle builder never moves the
windows to the host.  Training (GateUnits.py:61-113) is not part of the path
and stays with the reference; SGU1 (xgboost) stays on the host.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn

from . import _lib
from ._lib import check, ptr, stream_ptr

_KEYS = ("lstm.weight_ih_l0", "lstm.weight_hh_l0", "lstm.bias_ih_l0", "lstm.bias_hh_l0", "fc.weight", "fc.bias")


class SGU2Model(nn.Module):
    """GateUnits.py:42-54 (weights and state_dict layout)."""

    def __init__(self, input_size, hidden_size):
        super().__init__()
        self.lstm = nn.LSTM(input_size, hidden_size, batch_first=True)
        self.dropout = nn.Dropout(0.8)
        self.fc = nn.Linear(hidden_size, 1)

    def flat_weights(self) -> torch.Tensor:
        sd = self.state_dict()
        return torch.cat([sd[k].detach().reshape(-1).float().cpu() for k in _KEYS])


class StandardScaler3D:
    """utils/scaler.py: per-feature mean/std over (samples, time), + 1e-9."""

    def __init__(self, threshold=3.0):
        self.mean = None
        self.std = None
        self.threshold = threshold

    def fit(self, X):
        self.mean = np.mean(X, axis=(0, 1), keepdims=True)
        self.std = np.std(X, axis=(0, 1), keepdims=True) + 1e-9

    def transform(self, X):
        if self.mean is None or self.std is None:
            raise ValueError("Scaler has not been fitted yet.")
        return (X - self.mean) / self.std

    def fit_transform(self, X):
        self.fit(X)
        return self.transform(X)


class SGU2:
    """GateUnits.py:56-136 (inference side)."""

    def __init__(self, input_size=1, hidden_size=10, device="cpu"):
        if input_size != 1:
            raise ValueError("SGU2 windows carry one feature (HFTLoader.py:165-169)")
        self.device = torch.device(device)
        self.hidden_size = hidden_size
        self.model = SGU2Model(input_size, hidden_size)
        self.best_state = None
        self._w = None

    def _weights(self, dev):
        w = self.model.flat_weights()
        if self._w is None or self._w.device != dev or not torch.equal(self._w.cpu(), w):
            self._w = w.to(dev)
        return self._w

    def predict_device(self, X: torch.Tensor, scaler=None, out: torch.Tensor | None = None) -> torch.Tensor:
        """Windows [n, T, 1] (or [n, T]) float32 on the device -> float32 [n]
        (scaler: a fitted StandardScaler3D, applied in the kernel)."""
        _lib.require_gpu()
        L = _lib.load()
        X = X.contiguous()
        if X.dtype != torch.float32 or X.device.type != "cuda":
            raise TypeError("predict_device needs float32 windows on the device")
        n, T = int(X.shape[0]), int(X.shape[1]) if X.dim() > 1 else 0
        dev = X.device
        if out is None:
            out = torch.empty(max(n, 1), dtype=torch.float32, device=dev)
        m = s = None
        if scaler is not None:
            if np.asarray(scaler.mean).size != 1:
                raise ValueError("SGU2 windows carry one feature")
            m = torch.tensor(np.asarray(scaler.mean, np.float32).reshape(1), device=dev)
            s = torch.tensor(np.asarray(scaler.std, np.float32).reshape(1), device=dev)
        check(L.sgmm_sgu2_forward(ptr(self._weights(dev)), self.hidden_size, ptr(X), n, T, ptr(m), ptr(s),
                                  ptr(out), stream_ptr()), "sgmm_sgu2_forward")
        return out[:n]

    def predict(self, X):
        """GateUnits.py:116-120: numpy windows [n, T, 1] -> float32 [n, 1]."""
        X_t = torch.tensor(np.asarray(X), dtype=torch.float32).to("cuda")
        return self.predict_device(X_t).reshape(-1, 1).cpu().numpy()

    def train(self, *a, **k):
        raise NotImplementedError("SGU2 training (GateUnits.py:61-113) is not part of the GPU path; "
                                  "train with the reference and load() the checkpoint")

    def save(self, path):
        torch.save(self.model.state_dict(), path)

    def load(self, path):
        self.model.load_state_dict(torch.load(path, map_location="cpu", weights_only=True))
        self.model.eval()
        print(f"SGU2 model loaded from {path} and set to eval mode.")
