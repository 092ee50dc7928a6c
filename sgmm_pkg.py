"""Import helper: the package directory name has hyphens, so it is loaded by
path and registered as ``sgmm_amd``."""
import importlib.util
import sys
from pathlib import Path

PKG_NAME = "sgmm_amd"
PKG_DIR = Path(__file__).resolve().parent / "deep-reinforcement-learning-based-signal-gated-market-making_amd"


def load():
    if PKG_NAME in sys.modules:
        return sys.modules[PKG_NAME]
    spec = importlib.util.spec_from_file_location(PKG_NAME, PKG_DIR / "__init__.py",
                                                  submodule_search_locations=[str(PKG_DIR)])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[PKG_NAME] = mod
    try:
        spec.loader.exec_module(mod)
    except BaseException:
        sys.modules.pop(PKG_NAME, None)
        raise
    return mod


def build(force=False):
    spec = importlib.util.spec_from_file_location("_sgmm_build", PKG_DIR / "build.py")
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m.build_library(force=force)
