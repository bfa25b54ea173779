// fp_probe.hip -- exhaustive / randomized checks of the correctly rounded fp32 sqrt and divide
// fast paths the FedOPT kernels use (adapt_vec, flame_amd/csrc/fedagg.hip), against the
// general sequences LLVM emits for __builtin_sqrtf / __fdiv_rn, on the MI355X itself.
//
//   probe_sqrt(lo, hi, v, out): every fp32 bit pattern in [lo, hi): v=0 sqrt_rn (shipped), v=1
//                               v_sqrt_f32 alone, 2 sqrt_fix, 3 sqrt_rsq2 -- vs __builtin_sqrtf
//   probe_rcp(lo, hi, v, out):  every b in [lo, hi): v=0 v_rcp_f32, v=1 rcp_rn -- vs __fdiv_rn(1, b)
//   probe_div(seed, n, w, out): n counter-drawn (a, b) pairs: div_rn vs __fdiv_rn(a, b)
//   probe_den(lo, hi, tau, out): every v in [lo, hi): RN(sqrt_rn(v) + tau) vs RN(sqrtf(v) + tau)
//   probe_bf16_sqrt / _den / _div: the bf16 step's v_sqrt_f32 and num * v_rcp_f32(den) under the
//                               bf16 rounding, on every bf16 operand (adapt_vec_bf16)
// out[0] = mismatches, out[1..2] = the first mismatching operands (bits), out[3..4] = results.
// Built by tools/fp_probe.py (hipcc, same flags as the product library).
#include <hip/hip_runtime.h>
#include <cstdint>

#include "../flame_amd/csrc/fastmath.h"

namespace {

// exploratory sqrt candidates (not shipped): v_sqrt_f32 alone; LLVM's one-ulp correction of it
// without its denormal scaling; the rsq Newton step with y refined first
__device__ __forceinline__ float sqrt_hw(float x) { return __builtin_amdgcn_sqrtf(x); }
__device__ __forceinline__ float sqrt_fix(float x) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sd = __uint_as_float(__float_as_uint(s) - 1u);
    const float su = __uint_as_float(__float_as_uint(s) + 1u);
    const float rd = __builtin_fmaf(-sd, s, x);
    const float ru = __builtin_fmaf(-su, s, x);
    float r = rd <= 0.f ? sd : s;
    return ru > 0.f ? su : r;
}
__device__ __forceinline__ float sqrt_rsq2(float x) {
    const float y = __builtin_amdgcn_rsqf(x);
    const float s = x * y;
    const float h = 0.5f * y;
    const float e = __builtin_fmaf(-s, h, 0.5f);
    const float s1 = __builtin_fmaf(s, e, s);
    const float h1 = __builtin_fmaf(h, e, h);
    const float r = __builtin_fmaf(-s1, s1, x);
    return __builtin_fmaf(r, h1, s1);
}

__device__ void report(unsigned long long* out, uint32_t a, uint32_t b, uint32_t got, uint32_t want) {
    unsigned long long n = atomicAdd(out, 1ull);
    if (n == 0) {
        out[1] = a;
        out[2] = b;
        out[3] = got;
        out[4] = want;
    }
}

__global__ void sqrt_kernel(uint64_t lo, uint64_t hi, int variant, unsigned long long* out) {
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
    for (uint64_t i = lo + blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < hi; i += stride) {
        const float x = __uint_as_float(static_cast<uint32_t>(i));
        const float want = __builtin_sqrtf(x);
        const float got = variant == 0 ? flame_fm::sqrt_rn(x) : variant == 1 ? sqrt_hw(x)
                        : variant == 2 ? sqrt_fix(x) : sqrt_rsq2(x);
        if (__float_as_uint(got) != __float_as_uint(want))
            report(out, static_cast<uint32_t>(i), 0, __float_as_uint(got), __float_as_uint(want));
    }
}

__global__ void rcp_kernel(uint64_t lo, uint64_t hi, int variant, unsigned long long* out) {
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
    for (uint64_t i = lo + blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < hi; i += stride) {
        const float b = __uint_as_float(static_cast<uint32_t>(i));
        const float want = __fdiv_rn(1.0f, b);
        const float got = variant == 0 ? __builtin_amdgcn_rcpf(b) : flame_fm::rcp_rn(b);
        if (__float_as_uint(got) != __float_as_uint(want))
            report(out, static_cast<uint32_t>(i), 0, __float_as_uint(got), __float_as_uint(want));
    }
}

__device__ __forceinline__ uint64_t mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

// Counter-drawn (a, b).  wide = 0: the operands adapt_vec admits to the fast divide -- b in
// [2^-20, 2^40], a = +-0 (1/16 of the draws) or 2^-85 <= |a| <= 2^100, uniform exponents and
// mantissas, both signs of a; must match bit for bit.  wide = 1: a over every finite value
// (zeros, subnormals) and b in [2^-60, 2^66] (informational: outside the admitted range).
__global__ void div_kernel(uint64_t seed, uint64_t n, int wide, unsigned long long* out) {
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
    for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n; i += stride) {
        const uint64_t r = mix(seed * 0x9e3779b97f4a7c15ull + i);
        const uint32_t am = static_cast<uint32_t>(r) & 0x807fffffu;          // sign + mantissa
        const uint32_t bm = static_cast<uint32_t>(r >> 32) & 0x7fffffu;
        uint32_t ea, eb;
        uint32_t bmm = bm;
        if (wide == 2) {
            // the admitted range's corners: |a| in [2^-85, 2^-83) over b in [2^39, 2^40],
            // and |a| in [2^99, 2^100] over b in [2^-20, 2^-19) -- quotients down to 2^-125, where
            // Markstein's residual r * y is subnormal, and up to 2^120
            const uint32_t k = static_cast<uint32_t>(r >> 62);
            if (k < 2) {
                ea = 42u + k;
                eb = (r >> 61) & 1 ? 166u : 167u;
                if (eb == 167u) bmm = 0u;                      // b = 2^40 exactly
            } else {
                ea = k == 2 ? 226u : 227u;
                eb = 107u;
            }
            const uint32_t aa = (ea == 227u) ? (am & 0x80000000u) : am;   // |a| = 2^100 exactly
            const float a = __uint_as_float(aa | (ea << 23));
            const float b = __uint_as_float((eb << 23) | bmm);
            const float want = __fdiv_rn(a, b);
            const float got = flame_fm::div_rn(a, b);
            if (__float_as_uint(got) != __float_as_uint(want))
                report(out, __float_as_uint(a), __float_as_uint(b), __float_as_uint(got), __float_as_uint(want));
            continue;
        }
        if (wide) {
            ea = static_cast<uint32_t>((r >> 23) & 0xff) % 255u;
            eb = 67u + static_cast<uint32_t>((r >> 55) % 194u);
        } else {
            ea = ((r >> 60) == 0) ? 0u : 42u + static_cast<uint32_t>((r >> 23) % 186u);
            eb = 107u + static_cast<uint32_t>((r >> 55) % 61u);
        }
        const uint32_t ab = (ea == 0 && !wide) ? (am & 0x80000000u) : (am | (ea << 23));
        const float a = __uint_as_float(ab);
        const float b = __uint_as_float((eb << 23) | bm);
        const float want = __fdiv_rn(a, b);
        const float got = flame_fm::div_rn(a, b);
        if (__float_as_uint(got) != __float_as_uint(want))
            report(out, ab, __float_as_uint(b), __float_as_uint(got), __float_as_uint(want));
    }
}

// The denominator adapt_vec forms from a v below sqrt_rn's exact range: sqrt(v) + tau.
__global__ void den_kernel(uint64_t lo, uint64_t hi, float tau, unsigned long long* out) {
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
    for (uint64_t i = lo + blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < hi; i += stride) {
        const float v = __uint_as_float(static_cast<uint32_t>(i));
        const float want = __fadd_rn(__builtin_sqrtf(v), tau);
        const float got = __fadd_rn(flame_fm::sqrt_rn(v), tau);
        if (__float_as_uint(got) != __float_as_uint(want))
            report(out, static_cast<uint32_t>(i), __float_as_uint(tau), __float_as_uint(got), __float_as_uint(want));
    }
}

// bf16 (adapt_vec_bf16 in fedagg.hip): the bf16 rounding of v_sqrt_f32(v) vs of the correctly
// rounded root, for every bf16 v with hi16 in [lo, hi).
__device__ __forceinline__ float rbf(float x) { return static_cast<float>(static_cast<__bf16>(x)); }
__global__ void bf16_sqrt_kernel(uint32_t lo, uint32_t hi, unsigned long long* out) {
    const uint32_t i = lo + blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= hi) return;
    const float v = __uint_as_float(i << 16);
    const float want = rbf(__builtin_sqrtf(v));
    const float got = rbf(__builtin_amdgcn_sqrtf(v));
    if (__float_as_uint(got) != __float_as_uint(want)) report(out, i << 16, 0, __float_as_uint(got), __float_as_uint(want));
}

// ... and of num * v_rcp_f32(den) vs of the correctly rounded quotient, for every bf16 num (hi16 =
// blockIdx.y * 256 + x) that the fp32 step's admission takes (+-0, 2^-85 <= |num| <= 2^100; all = 0)
// or every bf16 num but NaN (all = 1: what adapt_vec_half admits, FLAME_T_HALF_ADMIT), and every
// bf16 den with hi16 in [dlo, dhi) (den = RN(RN(sqrt v) + tau) lies in [2^-20, 2^40] on admitted
// lanes).
__global__ void bf16_div_kernel(uint32_t dlo, uint32_t dhi, int all, unsigned long long* out) {
    const uint32_t nb = (blockIdx.y * 256u + threadIdx.x) << 16;
    const float num = __uint_as_float(nb);
    const float an = __builtin_fabsf(num);
    if (all ? __builtin_isnan(num) : !(an == 0.f || (an >= 0x1p-85f && an <= 0x1p100f))) return;
    for (uint32_t d = dlo + blockIdx.x; d < dhi; d += gridDim.x) {
        const float den = __uint_as_float(d << 16);
        const float want = rbf(__fdiv_rn(num, den));
        const float got = rbf(__fmul_rn(num, __builtin_amdgcn_rcpf(den)));
        if (__float_as_uint(got) != __float_as_uint(want)) report(out, nb, d << 16, __float_as_uint(got), __float_as_uint(want));
    }
}

// ... and the denominator the step forms from it, RN_bf16(RN_bf16(sqrt v) + tau), for every bf16 v with
// hi16 in [lo, hi) (v_sqrt_f32 flushes subnormal inputs to a zero root: under tau >= 2^-20 the
// denominator is tau either way)
__global__ void bf16_den_kernel(uint32_t lo, uint32_t hi, float tau, unsigned long long* out) {
    const uint32_t i = lo + blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= hi) return;
    const float v = __uint_as_float(i << 16);
    const float want = rbf(__fadd_rn(rbf(__builtin_sqrtf(v)), tau));
    const float got = rbf(__fadd_rn(rbf(__builtin_amdgcn_sqrtf(v)), tau));
    if (__float_as_uint(got) != __float_as_uint(want)) report(out, i << 16, __float_as_uint(tau), __float_as_uint(got), __float_as_uint(want));
}

// fp16 (adapt_vec_half, FLAME_T_F16_PACKED / FLAME_T_F16_HWROOT): the pair rounding
// v_cvt_pk_f16_f32 against v_cvt_f16_f32 per element on every fp32 pattern, and the hardware root
// / quotient under the fp16 rounding against the correctly rounded ones, on every fp16 operand.
__device__ __forceinline__ uint16_t h16(float x) {
    asm volatile("" : "+v"(x));
    _Float16 v = static_cast<_Float16>(x);
    uint16_t b;
    __builtin_memcpy(&b, &v, 2);
    return b;
}
__device__ __forceinline__ float f16v(uint32_t bits) {
    const uint16_t b = static_cast<uint16_t>(bits);
    _Float16 v;
    __builtin_memcpy(&v, &b, 2);
    return static_cast<float>(v);
}
__device__ __forceinline__ float rh(float x) { return f16v(h16(x)); }

__global__ void f16_pack_kernel(uint64_t lo, uint64_t hi, unsigned long long* out) {
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
    for (uint64_t i = lo + blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < hi; i += stride) {
        const float x = __uint_as_float(static_cast<uint32_t>(i));
        const float y = __uint_as_float(static_cast<uint32_t>(i) ^ 0x5a5a5a5au);
        uint32_t p;
        asm("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(p) : "v"(x), "v"(y));
        const uint32_t want = static_cast<uint32_t>(h16(x)) | (static_cast<uint32_t>(h16(y)) << 16);
        if (p != want) report(out, static_cast<uint32_t>(i), __float_as_uint(y), p, want);
    }
}

__global__ void f16_sqrt_kernel(uint32_t lo, uint32_t hi, float tau, unsigned long long* out) {
    const uint32_t i = lo + blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= hi) return;
    const float v = f16v(i);
    float want, got;
    if (tau == 0.f) {
        want = rh(flame_fm::sqrt_rn(v));
        got = rh(__builtin_amdgcn_sqrtf(v));
    } else {
        want = rh(__fadd_rn(rh(flame_fm::sqrt_rn(v)), tau));
        got = rh(__fadd_rn(rh(__builtin_amdgcn_sqrtf(v)), tau));
    }
    if (__float_as_uint(got) != __float_as_uint(want)) report(out, i, __float_as_uint(tau), __float_as_uint(got), __float_as_uint(want));
}

__global__ void f16_div_kernel(uint32_t dlo, uint32_t dhi, unsigned long long* out) {
    const uint32_t nb = blockIdx.y * 256u + threadIdx.x;
    const float num = f16v(nb);
    if (!(__builtin_fabsf(num) <= 65504.f)) return;              // every finite fp16 num is admitted
    for (uint32_t d = dlo + blockIdx.x; d < dhi; d += gridDim.x) {
        const float den = f16v(d);
        const float want = rh(flame_fm::div_rn(num, den));
        const float got = rh(__fmul_rn(num, __builtin_amdgcn_rcpf(den)));
        if (__float_as_uint(got) != __float_as_uint(want)) report(out, nb, d, __float_as_uint(got), __float_as_uint(want));
    }
}

// the packed-fp16 chain body's root (FLAME_T_F16_HSQRT): v_sqrt_f16 on a packed pair (the same
// builtin the kernel uses, so the same v_sqrt_f16 / v_sqrt_f16_sdwa pair) against the correctly
// rounded fp16 root; pattern i in the low half, i ^ 0x0155 (masked to the range) in the high half
using h2p = __attribute__((ext_vector_type(2))) _Float16;
__global__ void f16_hsqrt_kernel(uint32_t lo, uint32_t hi, unsigned long long* out) {
    const uint32_t i = lo + blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= hi) return;
    const uint32_t j = lo + ((i - lo) ^ 0x0155u) % (hi - lo);
    const uint32_t pair = i | (j << 16);
    const h2p s = __builtin_elementwise_sqrt(__builtin_bit_cast(h2p, pair));
    const uint32_t got = __builtin_bit_cast(uint32_t, s);
    const uint32_t want = static_cast<uint32_t>(h16(flame_fm::sqrt_rn(f16v(i)))) |
                          (static_cast<uint32_t>(h16(flame_fm::sqrt_rn(f16v(j)))) << 16);
    if (got != want) report(out, i, j, got, want);
}

// the chain body's scalar products: v_fma_mix_f32(s, half, neg(0)) against the fp32 product of the
// widened half, bit for bit (signed zeros included; NaNs compared as NaN), every fp16 pattern x the
// scalars in ss[0 .. ns)
__global__ void f16_mix_kernel(const float* ss, int ns, unsigned long long* out) {
    const uint32_t x = blockIdx.x * blockDim.x + threadIdx.x;     // 0 .. 65535
    const uint32_t pair = x | ((x ^ 0x8001u) << 16);
    for (int k = 0; k < ns; ++k) {
        const float sv = ss[k];
        float lo, hi;
        asm volatile("v_fma_mix_f32 %0, %1, %2, neg(0) op_sel_hi:[0,1,0]" : "=v"(lo) : "v"(sv), "v"(pair));
        asm volatile("v_fma_mix_f32 %0, %1, %2, neg(0) op_sel:[0,1,0] op_sel_hi:[0,1,0]" : "=v"(hi) : "v"(sv), "v"(pair));
        const float wl = __fmul_rn(sv, f16v(x)), wh = __fmul_rn(sv, f16v(x ^ 0x8001u));
        const bool okl = __float_as_uint(lo) == __float_as_uint(wl) || (lo != lo && wl != wl);
        const bool okh = __float_as_uint(hi) == __float_as_uint(wh) || (hi != hi && wh != wh);
        if (!(okl && okh)) report(out, x, __float_as_uint(sv), __float_as_uint(okl ? hi : lo), __float_as_uint(okl ? wh : wl));
    }
}

// fp64 (the elementwise programs' fp64 keys): how often the compiler's a / b and sqrt(x) differ
// from flame_fm::ddiv_rn / dsqrt_rn (the exact-residual step), on counter-drawn operands with
// exponents in [-(span), span); the step itself is checked for the nearest-value property it rests
// on: no neighbour of the result has a strictly smaller residual (divide) / the result's squared
// midpoints bracket x (root) -- a violation is a FAIL, a difference from the compiler is counted.
__global__ void f64_kernel(uint64_t seed, uint64_t n, int span, int root, unsigned long long* out,
                           unsigned long long* diff) {
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
    for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n; i += stride) {
        const uint64_t r1 = mix(seed * 0x9e3779b97f4a7c15ull + 2 * i), r2 = mix(seed * 0x9e3779b97f4a7c15ull + 2 * i + 1);
        const int64_t ea = static_cast<int64_t>(r1 >> 52) % (2 * span) - span + 1023;
        const int64_t eb = static_cast<int64_t>(r2 >> 52) % (2 * span) - span + 1023;
        const double a = __longlong_as_double((static_cast<long long>(ea) << 52) | (r1 & 0x000fffffffffffffull) |
                                              (root ? 0ull : (r2 & 0x8000000000000000ull)));
        const double b = __longlong_as_double((static_cast<long long>(eb) << 52) | (r2 & 0x000fffffffffffffull));
        double raw, got;
        bool ok;
        if (root) {
            raw = __builtin_sqrt(a);
            got = flame_fm::dsqrt_rn(a);
            const double sp = flame_fm::dnext(got, true), sm = flame_fm::dnext(got, false);
            const double rr = __builtin_fma(-got, got, a);
            ok = a < 0x1p-900 || (rr <= got * (sp - got) && rr > -got * (got - sm));
        } else {
            raw = a / b;
            got = flame_fm::ddiv_rn(a, b);
            const double gp = flame_fm::dnext(got, true), gm = flame_fm::dnext(got, false);
            const double rg = __builtin_fabs(__builtin_fma(-got, b, a));
            ok = !flame_fm::dmid(got) || (rg <= __builtin_fabs(__builtin_fma(-gp, b, a)) &&
                                          rg <= __builtin_fabs(__builtin_fma(-gm, b, a)));
        }
        if (__double_as_longlong(raw) != __double_as_longlong(got)) atomicAdd(diff, 1ull);
        if (!ok) report(out, static_cast<uint32_t>(i), static_cast<uint32_t>(i >> 32),
                        static_cast<uint32_t>(__double_as_longlong(got)), static_cast<uint32_t>(__double_as_longlong(raw)));
    }
}

}  // namespace

extern "C" {

int probe_f64(uint64_t seed, uint64_t n, int span, int root, unsigned long long* out, unsigned long long* diff) {
    (void)hipMemset(out, 0, 5 * sizeof(unsigned long long));
    (void)hipMemset(diff, 0, sizeof(unsigned long long));
    f64_kernel<<<8192, 256>>>(seed, n, span, root, out, diff);
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}

int probe_f16_hsqrt(uint32_t lo, uint32_t hi, unsigned long long* out) {
    (void)hipMemset(out, 0, 5 * sizeof(unsigned long long));
    if (hi > lo) f16_hsqrt_kernel<<<(hi - lo + 255) / 256, 256>>>(lo, hi, out);
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}

int probe_f16_mix(const float* ss, int ns, unsigned long long* out) {
    (void)hipMemset(out, 0, 5 * sizeof(unsigned long long));
    f16_mix_kernel<<<256, 256>>>(ss, ns, out);
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}

int probe_f16_pack(uint64_t lo, uint64_t hi, unsigned long long* out) {
    (void)hipMemset(out, 0, 5 * sizeof(unsigned long long));
    f16_pack_kernel<<<16384, 256>>>(lo, hi, out);
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}

int probe_f16_sqrt(uint32_t lo, uint32_t hi, float tau, unsigned long long* out) {
    (void)hipMemset(out, 0, 5 * sizeof(unsigned long long));
    if (hi > lo) f16_sqrt_kernel<<<(hi - lo + 255) / 256, 256>>>(lo, hi, tau, out);
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}

int probe_f16_div(uint32_t dlo, uint32_t dhi, unsigned long long* out) {
    (void)hipMemset(out, 0, 5 * sizeof(unsigned long long));
    f16_div_kernel<<<dim3(512, 256), 256>>>(dlo, dhi, out);
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}

int probe_bf16_den(uint32_t lo, uint32_t hi, float tau, unsigned long long* out) {
    (void)hipMemset(out, 0, 5 * sizeof(unsigned long long));
    if (hi > lo) bf16_den_kernel<<<(hi - lo + 255) / 256, 256>>>(lo, hi, tau, out);
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}

int probe_bf16_sqrt(uint32_t lo, uint32_t hi, unsigned long long* out) {
    (void)hipMemset(out, 0, 5 * sizeof(unsigned long long));
    if (hi > lo) bf16_sqrt_kernel<<<(hi - lo + 255) / 256, 256>>>(lo, hi, out);
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}

int probe_bf16_div(uint32_t dlo, uint32_t dhi, int all, unsigned long long* out) {
    (void)hipMemset(out, 0, 5 * sizeof(unsigned long long));
    bf16_div_kernel<<<dim3(512, 256), 256>>>(dlo, dhi, all, out);
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}

int probe_sqrt(uint64_t lo, uint64_t hi, int variant, unsigned long long* out) {
    (void)hipMemset(out, 0, 5 * sizeof(unsigned long long));
    sqrt_kernel<<<8192, 256>>>(lo, hi, variant, out);
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}

int probe_rcp(uint64_t lo, uint64_t hi, int variant, unsigned long long* out) {
    (void)hipMemset(out, 0, 5 * sizeof(unsigned long long));
    rcp_kernel<<<8192, 256>>>(lo, hi, variant, out);
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}

int probe_div(uint64_t seed, uint64_t n, int wide, unsigned long long* out) {
    (void)hipMemset(out, 0, 5 * sizeof(unsigned long long));
    div_kernel<<<8192, 256>>>(seed, n, wide, out);
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}

int probe_den(uint64_t lo, uint64_t hi, float tau, unsigned long long* out) {
    (void)hipMemset(out, 0, 5 * sizeof(unsigned long long));
    den_kernel<<<8192, 256>>>(lo, hi, tau, out);
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}

}  // extern "C"
