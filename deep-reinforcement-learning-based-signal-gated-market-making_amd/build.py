"""Build libsgmm.so for gfx950 with hipcc (no cmake / ninja needed).

Each translation unit is compiled to an object in parallel, then linked.

-ffp-contract=off keeps the float64 FTPEnv arithmetic unfused (the reference
evaluates best_bid - off_b * tick as a multiply then a subtract,
market_env.py:30-31); the MLP's fused multiply-adds are explicit fmaf calls.
"""
from __future__ import annotations

import hashlib
import os
import subprocess
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
SOURCES = ["csrc/sgmm_capi.hip", "csrc/sgmm_rollout.hip", "csrc/sgmm_frontier.hip", "csrc/sgmm_ga.hip",
           "csrc/sgmm_bundle.hip", "csrc/sgmm_sgu2.hip"]
HEADERS = ["csrc/sgmm_device.h", "csrc/sgmm_internal.h", "csrc/sgmm_ga_device.h", "csrc/sgmm_rollout.h",
           "../include/sgmm.h"]
ARCH = os.environ.get("SGMM_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-Wall", f"--offload-arch={ARCH}"]


def build_library(force: bool = False, verbose: bool = False, extra_flags: list[str] | None = None,
                  out: Path | None = None) -> Path:
    out = Path(out) if out else PKG_DIR / "libsgmm.so"
    deps = [PKG_DIR / s for s in SOURCES + HEADERS]
    flags = FLAGS + list(extra_flags or [])
    tag = hashlib.sha1(" ".join([HIPCC, *flags]).encode()).hexdigest()[:10]
    # the flag set a library was linked with sits beside it (libsgmm.so.flags):
    # a library is up to date only for the same flags and newer than every source
    side = out.with_name(out.name + ".flags")
    if (not force and out.exists() and side.exists() and side.read_text().strip() == tag
            and all(out.stat().st_mtime >= d.stat().st_mtime for d in deps)):
        return out
    # objects are cached per flag set (build/ is git-ignored): a translation
    # unit is recompiled when it or any shared header is newer than its object
    obj_dir = PKG_DIR / "build" / tag
    obj_dir.mkdir(parents=True, exist_ok=True)
    objs = [obj_dir / (Path(s).stem + ".o") for s in SOURCES]
    hdr_mtime = max((PKG_DIR / h).stat().st_mtime for h in HEADERS)

    def compile_one(i: int) -> None:
        src = PKG_DIR / SOURCES[i]
        if (not force and objs[i].exists()
                and objs[i].stat().st_mtime >= max(src.stat().st_mtime, hdr_mtime)):
            return
        cmd = [HIPCC, *flags, "-c", "-o", str(objs[i]) + ".tmp", str(src)]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        os.replace(str(objs[i]) + ".tmp", objs[i])

    with ThreadPoolExecutor(max_workers=min(len(SOURCES), os.cpu_count() or 1)) as pool:
        list(pool.map(compile_one, range(len(SOURCES))))
    cmd = [HIPCC, *flags, "-shared", "-o", str(out) + ".tmp", *map(str, objs)]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(str(out) + ".tmp", out)
    side.write_text(tag + "\n")
    return out


if __name__ == "__main__":
    import argparse

    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--force", action="store_true", help="recompile every translation unit")
    ap.add_argument("--out", default=None, help="library path (default: the in-tree libsgmm.so)")
    ap.add_argument("flags", nargs="*", help="extra compiler flags, e.g. -DSGMM_STAMPS (A/B variants)")
    a = ap.parse_args()
    print(build_library(force=a.force or a.out is None and not a.flags, verbose=True,
                        extra_flags=a.flags, out=a.out))
