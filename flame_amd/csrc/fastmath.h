// fastmath.h -- correctly rounded fp32 sqrt / reciprocal / divide for the operands the FedOPT
// step meets in practice (adapt_vec in fedagg.hip), cheaper than the general sequences LLVM
// emits for __builtin_sqrtf / __fdiv_rn, which also cover denormal, tiny, huge, inf and NaN
// operands (16 and 13 instructions, two of them quarter-rate, and none of them packable).
//
// Each function returns the SAME bits as the general sequence on the operands its admission
// predicate accepts, or (admits: v below 2^-96) bits that cannot change the step's results; the
// caller takes the general sequence for a lane where any operand is not admitted.
// tools/fp_probe.py checks this on the MI355X: exhaustively for sqrt_rn (every admitted x, and
// every v below 2^-96 through sqrt(v) + tau) and rcp_rn (every admitted b), and on counter-drawn
// admitted pairs for div_rn.
#pragma once
#include <hip/hip_runtime.h>

namespace flame_fm {

// RN(sqrt(x)) for x = +0 or 2^-96 <= x <= 2^78: from v_rsq_f32, s = x*y, h = y/2 and one
// Newton step on the root with the residual x - s*s exact by fma.  (v_sqrt_f32 alone is one ulp
// off on 15 % of the normals.)  rsq(+0) = +inf is clamped so that +0 maps to +0.
__device__ __forceinline__ bool sqrt_admits(float x) {
    return (__float_as_uint(x) == 0u) | ((x >= 0x1p-96f) & (x <= 0x1p78f));
}
__device__ __forceinline__ float sqrt_rn(float x) {
    // (a cheaper alternative, the seed of x + 2^-149 -- a packed add instead of a min -- fails at
    // +0: v_rsq_f32 flushes the subnormal, profiles/r05h_fp_probe_nudge.log)
    const float y = __builtin_fminf(__builtin_amdgcn_rsqf(x), 0x1p64f);
    const float s = x * y;
    const float h = 0.5f * y;
    const float r = __builtin_fmaf(-s, s, x);
    return __builtin_fmaf(r, h, s);
}

// RN(1/b) for 2^-20 <= b <= 2^40: the 1-ulp v_rcp_f32 and one Markstein correction.
__device__ __forceinline__ float rcp_rn(float b) {
    const float y0 = __builtin_amdgcn_rcpf(b);
    const float e = __builtin_fmaf(-b, y0, 1.0f);
    return __builtin_fmaf(e, y0, y0);
}

// RN(a/b) for 2^-20 <= b <= 2^40 and a = +-0 or 2^-85 <= |a| <= 2^100 (Markstein's theorem:
// y = RN(1/b), q0 = RN(a*y) within one ulp, the residual b*q0 - a exact, q = RN(q0 - r*y);
// 1/b, q0 and q are normal there).  The residual is taken negated so that a = +-0 gives +-0
// with a's sign, as IEEE division does.
__device__ __forceinline__ bool div_admits(float a) {
    const float aa = __builtin_fabsf(a);
    return (aa == 0.f) | ((aa >= 0x1p-85f) & (aa <= 0x1p100f));
}
__device__ __forceinline__ float div_rn(float a, float b) {
    const float y = rcp_rn(b);
    const float q0 = a * y;
    const float rn = __builtin_fmaf(b, q0, -a);
    return __builtin_fmaf(-rn, y, q0);
}

// What a lane's n elements need for sqrt_rn / div_rn to give adapt_vec's results bit for bit,
// with tau in [2^-20, 2^38] (checked by the caller), in three reductions:
//  * every v in [+0, 2^78] (the unsigned max of the bits; a sign, an inf or a NaN is above it).
//    On [2^-96, 2^78] and at +0 sqrt_rn is correctly rounded.  Below 2^-96 it is not, but only
//    den = RN(sqrt(v) + tau) uses it: both roots are under 2^-47 there (sqrt_rn's seed is
//    clamped at 2^64, so even a subnormal v that v_rsq_f32 flushes stays under 2^-60), far
//    below half an ulp of tau >= 2^-20, so den = tau either way -- and no lower bound on v costs
//    a compare;
//  * every eta*m +-0 or 2^-85 <= |num| <= 2^100: unsigned min of 2*bits-2 (drops the sign; +-0
//    wraps to the top) and the max of |num| (a NaN num passes it: the quotient is NaN on either
//    path, and NaN bits are not part of the contract).
// (A tiny eta*m could be admitted too while every current weight is >= 2^-30 -- c + q rounds to
// c for either quotient -- but that reduction adds 3-7 VALU instructions to the ~77 of a lane's
// 4-element step (ISA count), and only a weight whose average stays exactly equal to it decays m
// that far.)
template <int N>
__device__ __forceinline__ bool admits(const float (&v)[N], const float (&num)[N]) {
    uint32_t vhi = 0u, nlo = 0xffffffffu;
    float nhi = 0.f;
#pragma unroll
    for (int j = 0; j < N; ++j) {
        vhi = max(vhi, __float_as_uint(v[j]));
        nlo = min(nlo, (__float_as_uint(num[j]) << 1) - 2u);
        nhi = fmaxf(nhi, __builtin_fabsf(num[j]));
    }
    return (vhi <= 0x66800000u) & (nhi <= 0x1p100f) & (nlo >= (0x15000000u << 1) - 2u);
}

// The parts of admits the 16-bit steps need (adapt_vec_half in fedagg.hip): v in [+0, 2^78]
// (the root's and den's range), and a finite |num| <= 2^100 (a NaN passes: its quotient is NaN on
// either path) for fp16's div_rn, whose other bound, |num| >= 2^-85 or +-0, every fp16 value meets.
template <int N>
__device__ __forceinline__ bool admits_v(const float (&v)[N]) {
    uint32_t vhi = 0u;
#pragma unroll
    for (int j = 0; j < N; ++j) vhi = max(vhi, __float_as_uint(v[j]));
    return vhi <= 0x66800000u;
}
template <int N>
__device__ __forceinline__ bool admits_finite(const float (&num)[N]) {
    float nhi = 0.f;
#pragma unroll
    for (int j = 0; j < N; ++j) nhi = fmaxf(nhi, __builtin_fabsf(num[j]));
    return nhi <= 0x1p100f;
}

// fp64 divide and root correctly rounded, for the elementwise programs' fp64 keys (torch-CPU's
// are IEEE double ops): the compiler's sequences, then one exact-residual step.
//  * divide: of q = a / b and its two neighbours, the one with the smallest |a - c * b| (one fma
//    each, exact while a, b and q stay inside [2^-960, 2^960] in magnitude -- outside, q as the
//    compiler gives it), a tie to the even significand: |a - c b| = |b| |a / b - c|;
//  * root: s moves up iff x - s^2 > s * (s+ - s), down iff x - s^2 <= -s * (s - s-) -- x against
//    the squares of the two midpoints (x - s^2 is exact and a multiple of ulp(s)^2, so the ulp^2/4
//    terms never decide; a root is never a midpoint); x below 2^-900 is scaled by 2^1000 first.
// tools/fp_probe.py counts how often the compiler's results needed the step.
// the neighbours of a finite nonzero double toward +inf / -inf (its bits +-1)
__device__ __forceinline__ double dnext(double x, bool up) {
    const long long b = __double_as_longlong(x);
    return __longlong_as_double((x > 0.0) == up ? b + 1 : b - 1);
}
__device__ __forceinline__ bool dmid(double x) {
    const double ax = __builtin_fabs(x);
    return ax >= 0x1p-960 && ax <= 0x1p960;
}
__device__ __forceinline__ double ddiv_rn(double a, double b) {
    const double q = a / b;
    if (!(dmid(a) && dmid(b) && dmid(q))) return q;
    const double qp = dnext(q, true), qm = dnext(q, false);
    const double r = __builtin_fabs(__builtin_fma(-q, b, a)), rp = __builtin_fabs(__builtin_fma(-qp, b, a)),
                 rm = __builtin_fabs(__builtin_fma(-qm, b, a));
    auto odd = [](double x) { return (__double_as_longlong(x) & 1) != 0; };
    double best = q, rb = r;
    if (rp < rb || (rp == rb && odd(best))) { best = qp; rb = rp; }
    if (rm < rb || (rm == rb && odd(best))) { best = qm; rb = rm; }
    return best;
}
__device__ __forceinline__ double dsqrt_core(double x) {     // 2^-900 <= x < inf
    const double s = __builtin_sqrt(x);
    const double sp = dnext(s, true), sm = dnext(s, false);                  // s > 0
    const double r = __builtin_fma(-s, s, x);
    if (r > s * (sp - s)) return sp;
    if (r <= -s * (s - sm)) return sm;
    return s;
}
__device__ __forceinline__ double dsqrt_rn(double x) {
    if (!(x > 0.0) || !__builtin_isfinite(x)) return __builtin_sqrt(x);      // +-0, negatives, NaN, inf
    if (x < 0x1p-900) return dsqrt_core(x * 0x1p1000) * 0x1p-500;           // exact scalings
    return dsqrt_core(x);
}

}  // namespace flame_fm
