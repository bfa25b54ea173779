#!/usr/bin/env python3
"""Exhaustive / randomized bit checks of flame_amd/csrc/fastmath.h on the MI355X (see
tools/fp_probe.hip).  Prints one line per check with the mismatch count and the first
mismatching operands; exits non-zero when a variant the product uses mismatches.

    python tools/fp_probe.py --build          # here (hipcc, gfx950)
    python tools/fp_probe.py [--div-pairs N]  # on the GPU box
"""
import argparse
import ctypes
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
LIB = os.path.join(ROOT, "build", "probe", "libfp_probe.so")

NORMAL_LO, INF = 0x00800000, 0x7F800000


def f2b(x):
    import struct
    return struct.unpack("<I", struct.pack("<f", x))[0]


def build():
    from flame_amd import build as B
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    src = os.path.join(ROOT, "tools", "fp_probe.hip")
    subprocess.check_call([B.hipcc(), *B.HIPCC_FLAGS, "-o", LIB, src])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--div-pairs", type=float, default=2 ** 36)
    ap.add_argument("--lib", default=LIB)
    a = ap.parse_args()
    if a.build:
        return build()
    import torch
    L = ctypes.CDLL(a.lib)
    out = torch.zeros(5, dtype=torch.int64, device="cuda")
    p = ctypes.c_void_p(out.data_ptr())
    u64 = ctypes.c_uint64
    bad = 0

    def show(name, rc, must_be_exact):
        nonlocal bad
        o = out.cpu().tolist()
        ok = rc == 0 and (o[0] == 0 or not must_be_exact)
        bad += not ok
        first = "" if o[0] == 0 else f"; first: x={o[1]:#010x} y={o[2]:#010x} got={o[3]:#010x} want={o[4]:#010x}"
        print(f"{name}: rc={rc} mismatches={o[0]}{first}{'' if ok else '  <-- FAIL'}", flush=True)

    t = time.time()
    # sqrt: the admitted operands (+0, [2^-96, 2^78]) must match; the rest is informational
    SQ_LO, SQ_HI = f2b(2.0 ** -96), f2b(2.0 ** 78) + 1
    for v, nm in ((0, "sqrt_rn"), (1, "v_sqrt_f32 alone"), (2, "sqrt_fix"), (3, "sqrt_rsq2")):
        show(f"{nm} on +0", L.probe_sqrt(u64(0), u64(1), v, p), v == 0)
        show(f"{nm} on every x in [2^-96, 2^78]", L.probe_sqrt(u64(SQ_LO), u64(SQ_HI), v, p), v == 0)
        show(f"{nm} on every other normal", L.probe_sqrt(u64(NORMAL_LO), u64(SQ_LO), v, p), False)
        if v == 0:
            show(f"{nm} on (2^78, inf]", L.probe_sqrt(u64(SQ_HI), u64(INF + 1), v, p), False)
            show(f"{nm} on the subnormals", L.probe_sqrt(u64(1), u64(NORMAL_LO), v, p), False)
    for v, nm in ((0, "rcp v_rcp_f32 alone"), (1, "rcp_rn")):
        show(f"{nm} on every b in [2^-20, 2^40]", L.probe_rcp(u64(f2b(2.0 ** -20)), u64(f2b(2.0 ** 40) + 1), v, p),
             v == 1)
        show(f"{nm} on every normal b", L.probe_rcp(u64(NORMAL_LO), u64(INF), v, p), False)
    n = int(a.div_pairs)
    for seed in (1, 2):
        show(f"div_rn {n} admitted pairs (seed {seed})", L.probe_div(u64(seed), u64(n), 0, p), True)
    show(f"div_rn {n // 4} pairs over every finite a, b in [2^-60, 2^66] (outside the admitted range)",
         L.probe_div(u64(3), u64(n // 4), 1, p), False)
    show(f"div_rn {n // 4} pairs at the admitted corners (|a| near 2^-85 over b near 2^40, |a| near 2^100 "
         f"over b near 2^-20)", L.probe_div(u64(4), u64(n // 4), 2, p), True)
    # bf16 (adapt_vec_bf16): v_sqrt_f32 / num * v_rcp_f32 under the bf16 rounding, exhaustively
    u32 = ctypes.c_uint32
    L.probe_bf16_sqrt.argtypes = [u32, u32, ctypes.c_void_p]
    L.probe_bf16_div.argtypes = [u32, u32, ctypes.c_int, ctypes.c_void_p]
    L.probe_bf16_den.argtypes = [u32, u32, ctypes.c_float, ctypes.c_void_p]
    show("bf16: RN_bf16(v_sqrt_f32(v)) == RN_bf16(sqrt(v)) on bf16 v = +0", L.probe_bf16_sqrt(0, 1, p), True)
    show("bf16: RN_bf16(v_sqrt_f32(v)) == RN_bf16(sqrt(v)) on every normal bf16 v in [2^-126, 2^78]",
         L.probe_bf16_sqrt(0x0080, 0x6681, p), True)
    show("bf16: the same on the bf16 subnormals (v_sqrt_f32 flushes them: informational)",
         L.probe_bf16_sqrt(1, 0x0080, p), False)
    for tau in (2.0 ** -20, 1e-3, 1e-2, 0.1, 1.0, 2.0 ** 38):
        tb = float(torch.tensor(tau, dtype=torch.bfloat16))       # the step's tau is pre-rounded to bf16
        show(f"bf16: RN(RN(v_sqrt_f32(v)) + {tb:g}) == RN(RN(sqrt(v)) + {tb:g}) on every admitted bf16 v "
             f"(+0 .. 2^78, subnormals included)", L.probe_bf16_den(0, 0x6681, tb, p), True)
    show("bf16: v_sqrt_f32 on every other bf16 pattern (negative, > 2^78, inf, NaN; informational)",
         L.probe_bf16_sqrt(0x6681, 0x10000, p), False)
    show("bf16: RN_bf16(num * v_rcp_f32(den)) == RN_bf16(num / den) on every admitted bf16 num x every bf16 den "
         "in [2^-20, 2^40]", L.probe_bf16_div(0x3580, 0x5381, 0, p), True)
    show("bf16 (FLAME_T_HALF_ADMIT, shipped): the same on every bf16 num but NaN (zeros, the tiny and subnormal "
         "nums a decaying m reaches, huge, inf) x every bf16 den in [2^-20, 2^40]",
         L.probe_bf16_div(0x3580, 0x5381, 1, p), True)
    # fp16 (adapt_vec_half): the pair rounding on every fp32 pattern; the hardware root / quotient
    L.probe_f16_sqrt.argtypes = [u32, u32, ctypes.c_float, ctypes.c_void_p]
    L.probe_f16_div.argtypes = [u32, u32, ctypes.c_void_p]
    show("fp16: v_cvt_pk_f16_f32 == v_cvt_f16_f32 per half on every fp32 pattern (paired with x ^ 0x5a5a5a5a)",
         L.probe_f16_pack(u64(0), u64(1 << 32), p), True)
    show("fp16 (FLAME_T_F16_HWROOT, shipped): RN_f16(v_sqrt_f32(v)) == RN_f16(sqrt_rn(v)) on every non-negative "
         "finite fp16 v", L.probe_f16_sqrt(0, 0x7C00, 0.0, p), True)
    for tau in (2.0 ** -20, 1e-3, 1e-2, 0.1, 1.0):
        th = float(torch.tensor(tau, dtype=torch.float16))
        show(f"fp16 (shipped): RN(RN(v_sqrt_f32(v)) + {th:g}) == RN(RN(sqrt_rn(v)) + {th:g}) on every non-negative "
             f"finite fp16 v", L.probe_f16_sqrt(0, 0x7C00, th, p), True)
    show("fp16 (not shipped: the quotient stays div_rn): RN_f16(num * v_rcp_f32(den)) == RN_f16(div_rn(num, den)) on "
         "every finite fp16 num x every fp16 den in [2^-20, 65504]", L.probe_f16_div(0x0010, 0x7C00, p), False)
    # the packed-fp16 chain body (fedopt_chain_body_f16): v_sqrt_f16 on pairs, v_fma_mix_f32 products
    L.probe_f16_hsqrt.argtypes = [u32, u32, ctypes.c_void_p]
    show("fp16 (FLAME_T_F16_HSQRT, shipped): packed v_sqrt_f16 == RN_f16(sqrt_rn(v)) on every non-negative finite "
         "fp16 v (both halves)", L.probe_f16_hsqrt(0, 0x7C00, p), True)
    L.probe_f16_mix.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    g = torch.Generator().manual_seed(5)
    scal = torch.cat([torch.tensor([0.0, -0.0, 1.0, -1.0, 0.9, 0.1, 0.99, 0.01, 1e-2, 1 - 0.99, 4.0, -0.25, 2.0 ** -126,
                                    2.0 ** -149, 3e38, float("inf"), float("-inf")]),
                      (torch.randn(1007, generator=g) * torch.pow(2.0, torch.randint(-40, 40, (1007,), generator=g).float()))])
    scal_d = scal.float().to("cuda")
    show(f"fp16 (shipped): v_fma_mix_f32(s, half, neg(0)) == RN_f32(s * half) bit for bit on every fp16 pattern x "
         f"{scal.numel()} scalars (+-0, +-inf, subnormal, random)", L.probe_f16_mix(scal_d.data_ptr(), scal.numel(), p),
         True)
    # fp64 (flame_elementwise): the exact-residual step of ddiv_rn / dsqrt_rn, and how often it moved
    # the compiler's result
    L.probe_f64.argtypes = [u64, u64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    diff = torch.zeros(1, dtype=torch.int64, device="cuda")
    for root, span, nm in ((0, 60, "a / b"), (0, 1000, "a / b (wide exponents)"), (1, 60, "sqrt(x)"),
                           (1, 1022, "sqrt(x) (wide exponents)")):
        rc = L.probe_f64(u64(7 + root), u64(1 << 28), span, root, p, ctypes.c_void_p(diff.data_ptr()))
        show(f"fp64 {nm}: the corrected result is the nearest on {1 << 28} draws (the compiler's differed on "
             f"{int(diff.item())})", rc, True)
    # adapt_vec admits v below 2^-96 too: it only reaches sqrt(v) + tau (tau >= 2^-20)
    L.probe_den.argtypes = [u64, u64, ctypes.c_float, ctypes.c_void_p]
    for tau in (2.0 ** -20, 1e-3, 1e-2, 0.1, 1.0, 2.0 ** 38):
        show(f"sqrt_rn(v) + {tau:g} on every v in [+0, 2^-96)", L.probe_den(0, SQ_LO, tau, p), True)
    print(f"fp_probe: {time.time() - t:.1f} s, {bad} failing check(s)", flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
