"""Policy modules and the GA state, API-compatible with models/model.py of the
reference (TradingPolicy, AdversaryPolicy, NeuroEvolution).

These torch modules are the *weight containers* and the checkpoint format
(state_dict keys ``net.{0,2,4}.{weight,bias}`` as in model.py:8-15); their
genome vector (``get_weights``) is what the device rollout consumes.  The
population forward itself runs in the HIP kernels, not here.

Construction consumes the global torch RNG exactly like the reference
(nn.Linear default init, then orthogonal_(gain 0.9) / constant_(0.05),
model.py:17-21), so a run seeded with torch.manual_seed reproduces the
reference's initial masters and its ask() populations.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn


def genome_size(hidden: int) -> int:
    """Parameter count of TradingPolicy(hidden_dim=hidden): H*H + 7H + 2."""
    return hidden * hidden + 7 * hidden + 2


def hidden_from_genome(n: int) -> int:
    h = int(round((-7 + np.sqrt(49 - 4 * (2 - n))) / 2))
    if genome_size(h) != n:
        raise ValueError(f"{n} floats is not a TradingPolicy genome (H*H+7H+2)")
    return h


def genome_to_state_dict(genome, hidden: int) -> dict:
    """TradingPolicy state_dict (keys net.{0,2,4}.{weight,bias}) from a flat
    genome, without constructing a module (which would draw from the RNG)."""
    w = torch.as_tensor(genome, dtype=torch.float32).reshape(-1).cpu()
    H = hidden
    shapes = (("net.0.weight", (H, 3)), ("net.0.bias", (H,)), ("net.2.weight", (H, H)),
              ("net.2.bias", (H,)), ("net.4.weight", (2, H)), ("net.4.bias", (2,)))
    out, i = {}, 0
    for k, shp in shapes:
        n = int(np.prod(shp))
        out[k] = w[i:i + n].reshape(shp).clone()
        i += n
    if i != w.numel():
        raise ValueError(f"genome has {w.numel()} floats, H={H} needs {i}")
    return out


class TradingPolicy(nn.Module):
    """3 -> H -> H -> 2 ReLU MLP (models/model.py:5-36)."""

    def __init__(self, state_dim=3, action_dim=2, hidden_dim=32):
        super().__init__()
        self.net = nn.Sequential(
            nn.Linear(state_dim, hidden_dim), nn.ReLU(),
            nn.Linear(hidden_dim, hidden_dim), nn.ReLU(),
            nn.Linear(hidden_dim, action_dim))
        for layer in self.modules():
            if isinstance(layer, nn.Linear):
                nn.init.orthogonal_(layer.weight, gain=0.9)
                nn.init.constant_(layer.bias, 0.05)
        self.hidden_dim = hidden_dim
        self.eval()

    def forward(self, x):
        with torch.no_grad():
            return self.net(x)

    def get_weights(self) -> torch.Tensor:
        """Flat float32 genome in parameters() order."""
        return torch.cat([p.detach().reshape(-1) for p in self.parameters()]).clone()

    def set_weights(self, weights):
        w = torch.as_tensor(weights, dtype=torch.float32).reshape(-1)
        i = 0
        for p in self.parameters():
            n = p.numel()
            p.data.copy_(w[i:i + n].view_as(p).to(p.device))
            i += n


class AdversaryPolicy(nn.Module):
    """3 -> 12 -> 2 tanh perturbation policy (models/model.py:38-57).

    set_weights copies the LEADING 74 floats of whatever vector it is given;
    the reference's adversary evolver hands it 1250-float TradingPolicy
    genomes (model.py:63), and this aliasing is part of the semantics."""

    def __init__(self, input_size=3, hidden_size=12):
        super().__init__()
        self.fc = nn.Sequential(nn.Linear(input_size, hidden_size), nn.ReLU(),
                                nn.Linear(hidden_size, 2), nn.Tanh())

    def forward(self, x):
        return self.fc(x)

    def set_weights(self, weights):
        w = torch.as_tensor(weights, dtype=torch.float32).reshape(-1)
        i = 0
        for p in self.parameters():
            n = p.numel()
            p.data.copy_(w[i:i + n].view_as(p).to(p.device))
            i += n


class NeuroEvolution:
    """(1, lambda) neuroevolution state (models/model.py:59-76).

    ask() draws from the global torch CPU generator exactly as the reference
    does (bit-identical populations under torch.manual_seed).  DRLEngine
    generates populations on the GPU instead (rng="device") and uses this
    class only to hold the master and sigma."""

    def __init__(self, population_size=50, sigma=0.05, hidden_dim=32):
        self.pop_size = population_size
        self.sigma = sigma
        self.master_policy = TradingPolicy(hidden_dim=hidden_dim)

    def ask(self):
        master = self.master_policy.get_weights()
        return [master + torch.randn_like(master) * self.sigma for _ in range(self.pop_size)]

    def tell(self, population_weights, fitness_scores):
        best = int(np.argmax(fitness_scores))
        self.master_policy.set_weights(population_weights[best])
        return fitness_scores[best]
