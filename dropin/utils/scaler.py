"""Drop-in for the reference's utils/scaler.py (StandardScaler3D): the same
class, so a fitted float32 scaler lets load_signals_bundle apply it inside the
SGU2 kernel (bundle._fused_sgu2)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from _sgmm_path import sgmm  # noqa: E402
from sgmm_amd.gate_units import StandardScaler3D  # noqa: E402,F401
