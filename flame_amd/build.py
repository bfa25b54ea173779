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
import sysconfig

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
SRC = os.path.join(PKG, "csrc", "fedagg.hip")
HDR = os.path.join(ROOT, "include", "flame_amd.h")
DEPS = (SRC, HDR, os.path.join(PKG, "csrc", "fastmath.h"))
LIB = os.path.join(PKG, "libflame_amd.so")
# Sweep builds (tools/kernel_sweep.py, hier_sweep.py) compile SRC itself with -DFLAME_T_* overrides
# of its tunables into build/ab; diagnostic stamps are inserted into a copy by
# tools/sweep/htime.py.  Neither ever writes LIB.
ARCH = os.environ.get("FLAME_AMD_ARCH", "gfx950")
# host side: the restricted pickle VM of flame_amd.ingest (a CPython extension, plain gcc)
VM_SRC = os.path.join(PKG, "csrc", "pickle_vm.c")
VM_LIB = os.path.join(PKG, "_pickle_vm" + (sysconfig.get_config_var("EXT_SUFFIX") or ".so"))

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
    return any(os.path.getmtime(p) > t for p in DEPS)


def build_host(force: bool = False, verbose: bool = False) -> str:
    """The pickle VM extension (gcc, CPython headers)."""
    if not force and os.path.exists(VM_LIB) and os.path.getmtime(VM_LIB) >= os.path.getmtime(VM_SRC):
        return VM_LIB
    cmd = [os.environ.get("CC", "gcc"), "-O2", "-std=c11", "-shared", "-fPIC", "-Wall", "-Wextra", "-Werror",
           "-Wno-missing-field-initializers", f"-I{sysconfig.get_paths()['include']}", "-o", VM_LIB, VM_SRC]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    return VM_LIB


def build(force: bool = False, verbose: bool = False) -> str:
    """The product library: the fixed source, the fixed flags -- no ``-D`` overrides (a sweep
    build that forgot to restore a macro must never become the shipped kernel)."""
    build_host(force=force, verbose=verbose)
    if not force and not stale():
        return LIB
    cmd = [hipcc(), *HIPCC_FLAGS, "-o", LIB, SRC]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
