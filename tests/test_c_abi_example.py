"""The C ABI from plain C: examples/c_abi_fedavg.c compiles against include/flame_amd.h
(CPU) and, on the GPU, aggregates bit-identically to the reference arithmetic."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _build(tmp_path):
    from flame_amd import _native
    _native.lib()  # raises if the library is missing
    exe = str(tmp_path / "c_abi_fedavg")
    cmd = ["gcc", "-O2", "-std=c11", "-ffp-contract=off", "-Wall", "-Werror", "-D__HIP_PLATFORM_AMD__",
           "-I/opt/rocm/include", "-I", os.path.join(ROOT, "include"),
           os.path.join(ROOT, "examples", "c_abi_fedavg.c"),
           "-L", os.path.join(ROOT, "flame_amd"), "-lflame_amd", "-L/opt/rocm/lib", "-lamdhip64",
           f"-Wl,-rpath,{os.path.join(ROOT, 'flame_amd')}", "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return exe


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_c_example_compiles_against_header(tmp_path):
    assert os.path.exists(_build(tmp_path))


@pytest.mark.gpu
def test_c_example_runs_bitwise(tmp_path):
    exe = _build(tmp_path)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 / 100003 elements differ" in r.stdout
