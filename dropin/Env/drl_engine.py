"""Drop-in for the reference's Env/drl_engine.py (evaluate_individual,
DRLEngine): the population rollout and the GA loop run on the GPU through
libsgmm.so.  Same call signatures; DRLEngine accepts extra keyword-only
options (see sgmm_amd.drl_engine.DRLEngine)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from _sgmm_path import sgmm  # noqa: E402

evaluate_individual = sgmm.evaluate_individual
evaluate_population = sgmm.evaluate_population
DRLEngine = sgmm.DRLEngine
FTPEnv = sgmm.FTPEnv
TradingPolicy = sgmm.TradingPolicy
NeuroEvolution = sgmm.NeuroEvolution
AdversaryPolicy = sgmm.AdversaryPolicy
