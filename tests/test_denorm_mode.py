"""The built kernels keep fp32 denormals.

fastmath.h's div_rn is exact down to quotients near 2^-125 only because Markstein's correction
term r*y, subnormal there, is computed with denormals enabled; every bitwise test assumes one IEEE
rounding per op.  ``-ffast-math`` is refused by an ``#error`` in fedagg.hip, but
``-fgpu-flush-denormals-to-zero`` sets no macro -- so this test reads the mode the hardware will
run with from the code object itself: every kernel descriptor's COMPUTE_PGM_RSRC1
FLOAT_DENORM_MODE_32 field (bits 17:16; 3 = no flushing) in libflame_amd.so's gfx950 code object.
"""
import os
import struct
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "flame_amd", "libflame_amd.so")
LLVM = "/opt/rocm/lib/llvm/bin"


def _sections(data):
    shoff, = struct.unpack_from("<Q", data, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)
    secs = []
    for i in range(shnum):
        name, typ, flags, addr, off, size, link, info, align, entsize = struct.unpack_from(
            "<IIQQQQIIQQ", data, shoff + i * shentsize)
        secs.append(dict(name=name, type=typ, addr=addr, off=off, size=size, link=link, entsize=entsize))
    strtab = secs[shstrndx]

    def sname(o):
        s = data[strtab["off"] + o:]
        return s[:s.index(b"\0")].decode()
    for s in secs:
        s["sname"] = sname(s["name"])
    return secs


def kernel_descriptors(co: bytes):
    """{kernel name: COMPUTE_PGM_RSRC1} of an AMDGPU code object (ELF64)."""
    secs = _sections(co)
    symtab = next(s for s in secs if s["type"] == 2)
    strs = secs[symtab["link"]]
    out = {}
    for i in range(symtab["size"] // symtab["entsize"]):
        st_name, info, other, shndx, value, size = struct.unpack_from("<IBBHQQ", co, symtab["off"] + i * 24)
        nm = co[strs["off"] + st_name:]
        nm = nm[:nm.index(b"\0")].decode()
        if nm.endswith(".kd") and size == 64:
            sec = secs[shndx]
            kd = sec["off"] + value - sec["addr"]
            out[nm[:-3]] = struct.unpack_from("<I", co, kd + 48)[0]
    return out


def gfx950_code_object(tmp_path):
    fat = tmp_path / "fat.bin"
    subprocess.check_call([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", LIB, str(tmp_path / "x.so")])
    co = tmp_path / "k.co"
    subprocess.check_call([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                           "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"])
    return co.read_bytes()


@pytest.mark.skipif(not os.path.exists(LIB) or not os.path.exists(f"{LLVM}/clang-offload-bundler"),
                    reason="needs the built library and the ROCm LLVM tools")
def test_every_kernel_keeps_fp32_denormals(tmp_path):
    kds = kernel_descriptors(gfx950_code_object(tmp_path))
    assert len(kds) > 20, sorted(kds)
    assert any("fedopt_chain_kernel" in k for k in kds) and any("fedopt_kernel" in k for k in kds)
    flushed = {k: (r >> 16) & 3 for k, r in kds.items() if (r >> 16) & 3 != 3}
    assert not flushed, f"kernels built with fp32 denormal flushing (FLOAT_DENORM_MODE_32 != 3): {flushed}"


def test_fast_math_is_refused_at_compile_time():
    src = open(os.path.join(ROOT, "flame_amd", "csrc", "fedagg.hip")).read()
    assert "#error" in src and "__FAST_MATH__" in src and "__FINITE_MATH_ONLY__" in src
