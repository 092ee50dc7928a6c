"""Shared by the drop-in shims: put the repository root on sys.path and load
the package (its directory name has hyphens; sgmm_pkg registers it as
``sgmm_amd``)."""
import os
import sys

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)

import sgmm_pkg  # noqa: E402

sgmm = sgmm_pkg.load()
