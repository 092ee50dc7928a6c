"""Drop-in for the reference's models/model.py: TradingPolicy,
AdversaryPolicy, NeuroEvolution with the reference's module tree, state_dict
keys and RNG consumption (checkpoints load either way)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from _sgmm_path import sgmm  # noqa: E402

TradingPolicy = sgmm.TradingPolicy
AdversaryPolicy = sgmm.AdversaryPolicy
NeuroEvolution = sgmm.NeuroEvolution
