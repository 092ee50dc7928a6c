"""sgmm_amd -- MI355X-native population rollout for signal-gated market making.

Drop-in for the hot path of KAS-W/Deep-Reinforcement-Learning-Based-Signal-
Gated-Market-Making: FTPEnv (Env/market_env.py), TradingPolicy /
AdversaryPolicy / NeuroEvolution (models/model.py), evaluate_individual /
DRLEngine (Env/drl_engine.py); pipeline/agent_trainer.py then runs unchanged
on top of them (see dropin/ and INTEGRATION.md).  Compute runs in libsgmm.so (HIP, gfx950).

The directory name carries hyphens, so import it through the repository's
``sgmm_pkg.load()`` (registers it as ``sgmm_amd``), or put ``dropin/`` on
sys.path to resolve the reference's own module paths to this package.
"""
from .market_env import FTPEnv, FTPEnvBatch  # noqa: F401
from .model import (AdversaryPolicy, NeuroEvolution, TradingPolicy, genome_size,  # noqa: F401
                    genome_to_state_dict, hidden_from_genome)
from .rollout import (EnvConfig, EpisodeBatch, RolloutEngine, TickStore,  # noqa: F401
                      adversary_forward, normalize_signals, params_tensor, policy_forward)
from .drl_engine import DRLEngine, MultiDRLEngine, evaluate_individual, evaluate_population  # noqa: F401

__version__ = "0.1.0"
