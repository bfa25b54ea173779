// fp_probe.hip -- exhaustive / randomized checks of the correctly rounded fp32 sqrt and divide
// fast paths the FedOPT kernels use (adapt_vec, flame_amd/csrc/fedagg.hip), against the
// general sequences LLVM emits for __builtin_sqrtf / __fdiv_rn, on the MI355X itself.
//
//   probe_sqrt(lo, hi, v, out): every fp32 bit pattern in [lo, hi): v=0 sqrt_rn (shipped), v=1
//                               v_sqrt_f32 alone, 2 sqrt_fix, 3 sqrt_rsq2 -- vs __builtin_sqrtf
//   probe_rcp(lo, hi, v, out):  every b in [lo, hi): v=0 v_rcp_f32, v=1 rcp_rn -- vs __fdiv_rn(1, b)
//   probe_div(seed, n, w, out): n counter-drawn (a, b) pairs: div_rn vs __fdiv_rn(a, b)
//   probe_den(lo, hi, tau, out): every v in [lo, hi): RN(sqrt_rn(v) + tau) vs RN(sqrtf(v) + tau)
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

}  // namespace

extern "C" {

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
