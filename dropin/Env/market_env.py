"""Drop-in for the reference's Env/market_env.py: with ``dropin/`` ahead of the
reference root on sys.path, ``from Env.market_env import FTPEnv`` resolves
here (``Env`` is a namespace package in both trees, so the reference's other
Env modules -- recorder, benchmarks -- still import from the reference)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from _sgmm_path import sgmm  # noqa: E402

FTPEnv = sgmm.FTPEnv
FTPEnvBatch = sgmm.FTPEnvBatch
