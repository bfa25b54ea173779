"""Build the in-tree native library ``flame_amd/libflame_amd.so`` for gfx950.

Plain hipcc (no torch extension machinery): the library exposes only the C ABI
declared in ``include/flame_amd.h`` and is loaded with ctypes.

    python -m flame_amd.build           # build if stale
    python -m flame_amd.build --force   # rebuild
"""
from __future__ import annotations

import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
SRC = os.path.join(PKG, "csrc", "fedagg.hip")
HDR = os.path.join(ROOT, "include", "flame_amd.h")
LIB = os.path.join(PKG, "libflame_amd.so")
ARCH = os.environ.get("FLAME_AMD_ARCH", "gfx950")

HIPCC_FLAGS = [
    f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
    # one IEEE rounding per reference op: never contract a*b+c into an FMA
    "-ffp-contract=off", "-fno-fast-math",
    "-Wall", "-Wno-unused-function",
]


def hipcc() -> str:
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    cand = os.path.join(rocm, "bin", "hipcc")
    return cand if os.path.exists(cand) else "hipcc"


def stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(p) > t for p in (SRC, HDR))


def build(force: bool = False, verbose: bool = False, extra=None) -> str:
    if not force and not stale():
        return LIB
    cmd = [hipcc(), *HIPCC_FLAGS, *(extra or []), "-o", LIB, SRC]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
