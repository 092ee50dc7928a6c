"""Build libsgmm.so for gfx950 with hipcc (no cmake / ninja needed).

-ffp-contract=off keeps the float64 FTPEnv arithmetic unfused (the reference
evaluates best_bid - off_b * tick as a multiply then a subtract,
market_env.py:30-31); the MLP's fused multiply-adds are explicit fmaf calls.
"""
from __future__ import annotations

import os
import subprocess
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
SOURCES = ["csrc/sgmm_capi.hip", "csrc/sgmm_rollout.hip", "csrc/sgmm_ga.hip", "csrc/sgmm_bundle.hip",
           "csrc/sgmm_sgu2.hip"]
HEADERS = ["csrc/sgmm_device.h", "csrc/sgmm_internal.h", "csrc/sgmm_ga_device.h", "../include/sgmm.h"]
ARCH = os.environ.get("SGMM_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-Wall",
         f"--offload-arch={ARCH}"]


def build_library(force: bool = False, verbose: bool = False) -> Path:
    out = PKG_DIR / "libsgmm.so"
    deps = [PKG_DIR / s for s in SOURCES + HEADERS]
    if not force and out.exists() and all(out.stat().st_mtime >= d.stat().st_mtime for d in deps):
        return out
    cmd = [HIPCC, *FLAGS, "-o", str(out) + ".tmp", *[str(PKG_DIR / s) for s in SOURCES]]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(str(out) + ".tmp", out)
    return out


if __name__ == "__main__":
    print(build_library(force=True, verbose=True))
