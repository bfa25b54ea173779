// fedagg.hip -- CDNA4 (gfx950) kernels + C ABI for flame's server-side aggregation.
//
// Hot path: the weighted reduction of N client updates into
// one global model, restated from /root/reference/lib/python/flame/
//   optimizer/fedavg.py:79-104, optimizer/fedbuff.py:89-97,122-157,
//   optimizer/fedopt.py:102-129 (+ fedadam.py:33-35, fedyogi.py:34-36, fedadagrad.py:33-35).
//
// Design:
//   * HBM-read bound (≈1 flop per byte): no MFMA; every byte is read once.  LDS only holds
//     output blocks so their HBM writes go out as bursts (FedOPT, the hierarchy), or caps
//     residency at 2 workgroups per CU for long launches (HBM streams fastest there).
//   * One workgroup (256 lanes) owns one chunk of one segment; each lane owns
//     16 contiguous bytes of every client's update (dwordx4, non-temporal), so
//     every wave instruction is a 1 KiB fully-coalesced read.
//   * The client axis stays SEQUENTIAL in registers: per element the sum is
//     acc = round(acc + round(v_i * r_i)) in cache.iterkeys() order, exactly the
//     reference's torch-CPU op order -> bit-identical results.  Reordering the
//     fp32 client sum (tree / __shfl_down / split-K) breaks the 1e-6 contract
//     at N=1024, so it is not done.
//   * CU clients are unrolled per step so each lane has CU x 16 B loads in
//     flight (memory-level parallelism); client pointers and rates are
//     wave-uniform and come through the scalar cache.
//   * Built with -ffp-contract=off and explicit __f*_rn ops: no FMA contraction.
//   * Every host-side launch branch (which instantiation a launch takes) is counted
//     (flame_launch_branch_count) and pinned by a GPU oracle test.
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>

#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <cstdarg>
#include <type_traits>

#include "../../include/flame_amd.h"
#include "fastmath.h"

// One IEEE rounding per reference op, denormals kept (fastmath.h's div_rn proof and every bitwise
// test rest on it).  -ffast-math / -ffinite-math-only are refused here; the denormal mode of the
// built kernels (-fgpu-flush-denormals-to-zero sets no macro) is checked on the code object by
// tests/test_denorm_mode.py.
#if defined(__FAST_MATH__) || (defined(__FINITE_MATH_ONLY__) && __FINITE_MATH_ONLY__)
#error "fedagg.hip must not be built with -ffast-math / -ffinite-math-only"
#endif

namespace {

// Tunables, each chosen by an interleaved A/B sweep on MI355X.  The product build
// (flame_amd/build.py) passes no -D: these defaults ARE the shipped kernel.  The sweep tools
// (tools/hier_sweep.py, tools/chain_sweep.py, ...) build variants of THIS source with -DFLAME_T_*
// overrides into build/, so a sweep always measures the shipped code with one knob moved.
constexpr int kBlock = 256;          // lanes per workgroup of the reduction kernels
constexpr int kVPT = 1;              // 16-byte vectors per lane per client
#ifndef FLAME_T_CLIENT_UNROLL
#define FLAME_T_CLIENT_UNROLL 8
#endif
constexpr int kClientUnroll = FLAME_T_CLIENT_UNROLL;     // clients whose loads are issued together per lane (full residency)
#ifndef FLAME_T_CLIENT_UNROLL16
#define FLAME_T_CLIENT_UNROLL16 8
#endif
constexpr int kClientUnroll16 = FLAME_T_CLIENT_UNROLL16;   // the same for 16-bit dtypes (8 elements per lane vector)
// flame_agg_reduce, launches of >= kLoMinClients clients over >= kLoMinChunks chunks: 2 workgroups
// per CU (kLoLds of dynamic LDS, unused) with a client unroll of 3 (16-bit: 4) -- fewer loads in
// flight read HBM faster (C3: 14.90 -> 14.18 ms, 99 % of a region probe at that residency;
// profiles/r03ze_c3_sweep.log, r03zf_c3_sweep.log, r03zf_c3_bf16_sweep.log)
#ifndef FLAME_T_LO_UNROLL
#define FLAME_T_LO_UNROLL 3
#endif
constexpr int kLoUnroll = FLAME_T_LO_UNROLL;
#ifndef FLAME_T_LO_UNROLL16
#define FLAME_T_LO_UNROLL16 4
#endif
constexpr int kLoUnroll16 = FLAME_T_LO_UNROLL16;
#ifndef FLAME_T_LO_LDS
#define FLAME_T_LO_LDS 65536
#endif
constexpr int kLoLds = FLAME_T_LO_LDS;
// Below kLoBurstMaxClients clients the low-residency launch also holds kLoWGC chunks' outputs per
// workgroup in LDS and stores them in one burst: the short client streams of such rounds pay for
// every interleaved store.  Tiled slab, one process, bitwise (tools/kernel_sweep.py,
// profiles/r05s_lo_wgc_*.log, r05t_lo_wgc_*.log): fp32 x 25M, 64 clients 0.964 -> 0.909 ms, 128
// 1.843 -> 1.797, 256 3.594 -> 3.546, 512 equal, 1,024 +0.8 %; bf16 x 50M, 64 clients 1.028 ->
// 0.969 ms, 256 3.647 -> 3.621.  (A kernel-argument launch never holds 512 clients' pointers, so
// its low-residency launches always burst.)
#ifndef FLAME_T_LO_WGC
#define FLAME_T_LO_WGC 8
#endif
constexpr int kLoWGC = FLAME_T_LO_WGC;
#ifndef FLAME_T_LO_BURST_MAX_CLIENTS
#define FLAME_T_LO_BURST_MAX_CLIENTS 512
#endif
constexpr int kLoBurstMaxClients = FLAME_T_LO_BURST_MAX_CLIENTS;
// the dynamic LDS that, beside the kLoWGC chunks' held outputs (4 KiB each), still makes kLoLds per workgroup
constexpr int kLoHeld = kLoWGC > 1 ? kLoWGC * 4096 : 0;
constexpr int kLoDynLds = kLoLds > kLoHeld ? kLoLds - kLoHeld : 0;
#ifndef FLAME_T_LO_MIN_CLIENTS
#define FLAME_T_LO_MIN_CLIENTS 64
#endif
constexpr int kLoMinClients = FLAME_T_LO_MIN_CLIENTS;    // 64 x 100M fp32: 4.04 -> 3.90 ms (profiles/r03zn_c64_lomin.log)
#ifndef FLAME_T_LO_MIN_CHUNKS
#define FLAME_T_LO_MIN_CHUNKS 4096
#endif
constexpr int64_t kLoMinChunks = FLAME_T_LO_MIN_CHUNKS;
// FedOPT (fp32, >= 8 x 256 x kOptWGC chunks): kOptWGC chunks per workgroup, their avg/m/v/cur
// blocks held in LDS (16 KiB per chunk -> 2 workgroups per CU) and stored in one burst at the end,
// client unroll kOptUnroll (profiles/r02_fedopt_wgc_sweep.log, r03zf_c4_sweep.log, r03zg_c4_sweep.log)
#ifndef FLAME_T_OPT_WGC
#define FLAME_T_OPT_WGC 4
#endif
constexpr int kOptWGC = FLAME_T_OPT_WGC;
#ifndef FLAME_T_OPT_UNROLL
#define FLAME_T_OPT_UNROLL 3
#endif
constexpr int kOptUnroll = FLAME_T_OPT_UNROLL;
// hierarchy kernel: register store groups of kHB middles (16-bit client unroll kHierUnroll16);
// launches of >= kHLdsMinMids middles hold store groups of kHBL middles in LDS (4 KiB each per
// workgroup, 2 workgroups per CU) with a 16-bit unroll of kHierLdsUnroll16 (C5 shard 20.99 ->
// 19.51 ms, profiles/r02_hier_lds_sweep.log); one middle over >= 64 arrivals and >= 4,096 chunks
// (a FedBuff aggregator's fused scale_add): low residency, unroll 3 (profiles/r03zv_fedbuff_*.log)
#ifndef FLAME_T_HB
#define FLAME_T_HB 8
#endif
constexpr int kHB = FLAME_T_HB;
#ifndef FLAME_T_HIER_UNROLL16
#define FLAME_T_HIER_UNROLL16 4
#endif
constexpr int kHierUnroll16 = FLAME_T_HIER_UNROLL16;
#ifndef FLAME_T_HBL
#define FLAME_T_HBL 16
#endif
constexpr int kHBL = FLAME_T_HBL;
#ifndef FLAME_T_HIER_LDS_UNROLL16
#define FLAME_T_HIER_LDS_UNROLL16 6
#endif
constexpr int kHierLdsUnroll16 = FLAME_T_HIER_LDS_UNROLL16;
#ifndef FLAME_T_HLDS_MIN_MIDS
#define FLAME_T_HLDS_MIN_MIDS 16
#endif
constexpr int kHLdsMinMids = FLAME_T_HLDS_MIN_MIDS;
#ifndef FLAME_T_HLO_UNROLL
#define FLAME_T_HLO_UNROLL 3
#endif
constexpr int kHLoUnroll = FLAME_T_HLO_UNROLL;
#ifndef FLAME_T_HLO_MIN_CLIENTS
#define FLAME_T_HLO_MIN_CLIENTS 64
#endif
constexpr int kHLoMinClients = FLAME_T_HLO_MIN_CLIENTS;
#ifndef FLAME_T_HLO_MIN_CHUNKS
#define FLAME_T_HLO_MIN_CHUNKS 4096
#endif
constexpr int64_t kHLoMinChunks = FLAME_T_HLO_MIN_CHUNKS;
#ifndef FLAME_T_HLO_LDS_F32
#define FLAME_T_HLO_LDS_F32 65536
#endif
constexpr int kHLoLdsF32 = FLAME_T_HLO_LDS_F32;    // 2 workgroups per CU
#ifndef FLAME_T_HLO_LDS16
#define FLAME_T_HLO_LDS16 53248
#endif
constexpr int kHLoLds16 = FLAME_T_HLO_LDS16;     // 3 workgroups per CU
#ifndef FLAME_T_DYN_UNROLL
#define FLAME_T_DYN_UNROLL 4
#endif
constexpr int kDynUnroll = FLAME_T_DYN_UNROLL;
#ifndef FLAME_T_CHAIN_UNROLL
#define FLAME_T_CHAIN_UNROLL 16
#endif
constexpr int kChainUnroll = FLAME_T_CHAIN_UNROLL;     // eager FedOPT chain: client loads in flight per lane
#ifndef FLAME_T_CHAIN_UNROLL16
#define FLAME_T_CHAIN_UNROLL16 8
#endif
constexpr int kChainUnroll16 = FLAME_T_CHAIN_UNROLL16;
// fp32 chain: 16 client loads in flight per lane at 3 workgroups per CU (dynamic LDS as the cap):
// 1.453 -> 1.358 ms per 64 x 25M round against 8 at full residency, one process, bitwise
// (profiles/r05g_chain_ab.log); 16-bit chains keep 8 at full residency
#ifndef FLAME_T_CHAIN_LDS
#define FLAME_T_CHAIN_LDS 53248
#endif
constexpr int kChainLds = FLAME_T_CHAIN_LDS;           // dynamic LDS per fp32 workgroup (a residency cap)
// bf16 FedOPT step (adapt_vec) and eager-chain arrivals: two elements per packed fp32 instruction,
// one instruction per bf16 rounding, v_sqrt_f32 / v_rcp_f32 where the bf16 rounding absorbs their
// ulp; 0 = the generic per-element path (same bits, for A/B builds)
#ifndef FLAME_T_BF16_PACKED
#define FLAME_T_BF16_PACKED 1
#endif
constexpr bool kBf16Packed = FLAME_T_BF16_PACKED != 0;
// the same for fp16 (two elements per fp32 instruction, a pair rounded by one v_cvt_pk_f16_f32 and
// widened back by two converts); 0 = the generic per-element path
#ifndef FLAME_T_F16_PACKED
#define FLAME_T_F16_PACKED 1
#endif
constexpr bool kF16Packed = FLAME_T_F16_PACKED != 0;
// fp16 root: v_sqrt_f32 under the fp16 rounding (1; tools/fp_probe.py finds it equal to the
// correctly rounded root's on every finite fp16 v, and the step's denominator on every v for every
// tau it draws, profiles/r06l_fp_probe.log) or flame_fm::sqrt_rn, then the rounding (0).  The
// quotient stays flame_fm::div_rn: num * v_rcp_f32 differs on 10,528 fp16 pairs (ties of subnormal
// results, where an fp16 quotient has too few bits for the midpoint argument)
#ifndef FLAME_T_F16_HWROOT
#define FLAME_T_F16_HWROOT 1
#endif
constexpr bool kF16HwRoot = FLAME_T_F16_HWROOT != 0;
// fp16 eager chain (full, aligned chunks): base / current / m / v held as packed fp16 pairs, every
// fp16-by-fp16 op one v_pk_add_f16 / v_pk_mul_f16, every scalar product two v_fma_mix_f32 and a
// v_cvt_pk_f16_f32 (1; fedopt_chain_body_f16), or the fp32-register step (0); same bits
#ifndef FLAME_T_F16_NATIVE
#define FLAME_T_F16_NATIVE 1
#endif
constexpr bool kF16Native = FLAME_T_F16_NATIVE != 0;
// ... and its root: v_sqrt_f16 on the packed pair (1; tools/fp_probe.py: equal to the correctly
// rounded fp16 root on every fp16 v >= +0) or v_sqrt_f32 on the widened halves (0)
#ifndef FLAME_T_F16_HSQRT
#define FLAME_T_F16_HSQRT 1
#endif
constexpr bool kF16HalfRoot = FLAME_T_F16_HSQRT != 0;
// the 16-bit steps' fast-path admission (adapt_vec_half): 1 = only what their root / quotient need --
// v in [+0, 2^78] for both, and for fp16 (flame_fm::div_rn) a finite |num|: every nonzero finite
// fp16 value is >= 2^-24, inside div_rn's range, and the bf16 quotient num * v_rcp_f32 matches on
// every non-NaN bf16 num (tools/fp_probe.py) -- so a bf16 m decaying through [2^-133, 2^-85]
// (a weight whose average stops moving) no longer sends its lane down the general path;
// 0 = the fp32 step's admission (flame_fm::admits), for A/B builds
#ifndef FLAME_T_HALF_ADMIT
#define FLAME_T_HALF_ADMIT 1
#endif
constexpr bool kHalfAdmit = FLAME_T_HALF_ADMIT != 0;
// FedYogi's (1 - beta_2) d^2 * sign(v - d^2): sign as one ordered compare + bit-select (1) or as
// torch writes it, two compares and an integer difference (0); same bits
#ifndef FLAME_T_YOGI_SIGN
#define FLAME_T_YOGI_SIGN 1
#endif
constexpr bool kYogiSelect = FLAME_T_YOGI_SIGN != 0;
constexpr int kEwBlock = 256;  // elementwise kernels (scale-add, synth)

thread_local char g_err[512] = "";

int set_err(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_err(FLAME_EHIP, "%s: %s", what, hipGetErrorString(e));
    g_err[0] = 0;
    return FLAME_OK;
}

// ---------------------------------------------------------------- rounding helpers
__device__ __forceinline__ float bf16_round(float x) {
    // RNE fp32 -> bf16 -> fp32 (v_cvt_pk_bf16_f32 on gfx950)
    return static_cast<float>(static_cast<__bf16>(x));
}
__device__ __forceinline__ float bf16_to_f32(uint16_t b) {
    return __uint_as_float(static_cast<uint32_t>(b) << 16);
}
__device__ __forceinline__ uint16_t f32_to_bf16_exact(float x) {  // x already bf16-representable
    return static_cast<uint16_t>(__float_as_uint(x) >> 16);
}
// The same rounding with the result left where fp32 wants it (bits = bf16 << 16): ONE
// v_cvt_pk_bf16_f32 whose low half converts +0, instead of the convert into the low half and the
// shift up that bf16_round compiles to -- the same instruction, so the same bits (NaNs included).
// Never applied to a transcendental's result: gfx950 needs a wait state before a VALU reads a
// v_sqrt / v_rcp / v_rsq result, and the compiler does not insert it ahead of inline asm (those
// roundings use bf16_round).
__device__ __forceinline__ float bf16_rnd1(float x) {
    float r;
    asm("v_cvt_pk_bf16_f32 %0, 0, %1" : "=v"(r) : "v"(x));
    return r;
}
using f2 = __attribute__((ext_vector_type(2))) float;    // v_pk_{mul,add,fma}_f32 operands
__device__ __forceinline__ f2 bf16_rnd2(f2 x) { return f2{bf16_rnd1(x.x), bf16_rnd1(x.y)}; }
__device__ __forceinline__ f2 splat2(float x) { return f2{x, x}; }
// The empty asm pins x as an fp32 VGPR value: without it the backend folds
// fptrunc(fmul(a, r)) into v_fma_mixlo_f16, which rounds the exact product to
// fp16 ONCE, while torch rounds the fp32 product to fp16 (two roundings; they
// differ for an fp32 rate).
__device__ __forceinline__ float f16_round(float x) {
    asm volatile("" : "+v"(x));
    return static_cast<float>(static_cast<_Float16>(x));
}
__device__ __forceinline__ float f16_to_f32(uint16_t h) {
    _Float16 v;
    __builtin_memcpy(&v, &h, 2);
    return static_cast<float>(v);
}
__device__ __forceinline__ uint16_t f32_to_f16_bits(float x) {
    asm volatile("" : "+v"(x));
    _Float16 v = static_cast<_Float16>(x);
    uint16_t h;
    __builtin_memcpy(&h, &v, 2);
    return h;
}
// A pair RNE-rounded to fp16 and widened back: ONE v_cvt_pk_f16_f32 (the same conversion as
// f16_round's v_cvt_f16_f32, per half; inline asm, so the backend cannot fold a product into a
// single-rounding v_fma_mix) and two exact widening converts (the high half by SDWA).  Never
// applied to a transcendental's result (see bf16_rnd1).
__device__ __forceinline__ f2 f16_rnd2(f2 x) {
    uint32_t p;
    asm("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(p) : "v"(x.x), "v"(x.y));
    return f2{f16_to_f32(static_cast<uint16_t>(p)), f16_to_f32(static_cast<uint16_t>(p >> 16))};
}

// fp16 pairs kept packed (the fp16 eager chain, FLAME_T_F16_NATIVE).  An op on two fp16 values
// rounded once to fp16 (v_pk_add_f16 / v_pk_mul_f16) equals torch-CPU's op in fp32 rounded to fp16:
// a product of two 11-bit significands is exact in fp32, and for a sum, square root or quotient
// fp32's 24 bits are >= 2p + 2 for p = 11, so rounding to fp32 first never changes the fp16
// rounding (Figueroa's double-rounding theorem).  A Python-scalar operand (beta, eta, a rate) is
// fp32 (24 bits), so those products go through fp32: smul_h2.
using h2 = __attribute__((ext_vector_type(2))) _Float16;
using us2 = __attribute__((ext_vector_type(2))) unsigned short;
__device__ __forceinline__ h2 h2_of(uint32_t u) { return __builtin_bit_cast(h2, u); }
__device__ __forceinline__ uint32_t u_of(h2 h) { return __builtin_bit_cast(uint32_t, h); }
__device__ __forceinline__ f2 widen_h2(uint32_t u) {
    const h2 h = h2_of(u);
    return f2{static_cast<float>(h.x), static_cast<float>(h.y)};
}
// RN16(RN32(s * x)) of a pair: two v_fma_mix_f32 (a half widened exactly inside the instruction;
// s * x + neg(0) = s * x + (-0) rounded once is the fp32 product, signed zeros included) and one v_cvt_pk_f16_f32 --
// instead of two widening converts, a v_pk_mul_f32, the rounding and two more widening converts.
// (lo, hi: the two fp32 products before the fp16 rounding)
__device__ __forceinline__ uint32_t smul_h2(float s, uint32_t x, float& lo, float& hi) {
    uint32_t r;
    asm("v_fma_mix_f32 %0, %1, %2, neg(0) op_sel_hi:[0,1,0]" : "=v"(lo) : "s"(s), "v"(x));
    asm("v_fma_mix_f32 %0, %1, %2, neg(0) op_sel:[0,1,0] op_sel_hi:[0,1,0]" : "=v"(hi) : "s"(s), "v"(x));
    asm("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(r) : "v"(lo), "v"(hi));
    return r;
}
__device__ __forceinline__ uint32_t smul_h2(float s, uint32_t x) {
    float lo, hi;
    return smul_h2(s, x, lo, hi);
}
// flame_fm::div_rn(num, den) with the numerator an fp16 half of x (HI: the high one): q0 = y * num
// as one v_fma_mix_f32 (the widening inside it), the residual's -num folded the same way by the
// compiler -- the same four roundings as div_rn on the widened value.  y is rcp_rn's fma result,
// never a v_rcp_f32 result, so no transcendental feeds the inline asm.
template <int HI>
__device__ __forceinline__ float div_rn_h(uint32_t x, float den) {
    const float y = flame_fm::rcp_rn(den);
    float q0;
    if constexpr (HI) asm("v_fma_mix_f32 %0, %1, %2, neg(0) op_sel:[0,1,0] op_sel_hi:[0,1,0]" : "=v"(q0) : "v"(y), "v"(x));
    else asm("v_fma_mix_f32 %0, %1, %2, neg(0) op_sel_hi:[0,1,0]" : "=v"(q0) : "v"(y), "v"(x));
    const float a = static_cast<float>(HI ? h2_of(x).y : h2_of(x).x);
    const float rn = __builtin_fmaf(den, q0, -a);
    return __builtin_fmaf(-rn, y, q0);
}
// RN16 of an fp32 pair, packed (never on a transcendental's result, see bf16_rnd1)
__device__ __forceinline__ uint32_t pk_h2(f2 x) {
    uint32_t r;
    asm("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(r) : "v"(x.x), "v"(x.y));
    return r;
}
// torch.sign of an fp16 pair as FedYogi's t * sign(x) uses it: +-1 for a nonzero x, +0 for +-0.
// x + 0 turns -0 into +0; x * 65504 * 65504 carries the smallest subnormal (2^-24) past 1 and
// overflows the rest to inf; the clamp to [-1, 1] keeps +-1 / +0.  A NaN x clamps to +1 (minNum),
// not to torch's 0 -- but a NaN x = v - d^2 means v or d^2 is a NaN (t * sign is then NaN either
// way) or v = d^2 = +inf (t = inf: inf * 0 and inf - inf * 1 are both NaN), so v's new value is a
// NaN on both ways.
__device__ __forceinline__ h2 sign_h2(h2 x) {
    const h2 z = x + h2{0, 0};
    const h2 big = (z * h2{65504, 65504}) * h2{65504, 65504};
    return __builtin_elementwise_max(__builtin_elementwise_min(big, h2{1, 1}), h2{-1, -1});
}

// ---------------------------------------------------------------- dtype traits
// T: storage type; A: register accumulator type; EPT: elements per 16-byte lane vector.
// tmp(v, r) = the reference's `tmp = (v * rate).to(v.dtype)`; add(a, t) = `agg += tmp`.
template <int DT> struct Tr;

template <> struct Tr<FLAME_F32> {
    using T = float; using A = float; static constexpr int EPT = 4;
    __device__ static A ld(T x) { return x; }
    __device__ static T st(A a) { return a; }
    __device__ static A tmp(T v, float r, double) { return __fmul_rn(v, r); }
    __device__ static A add(A a, A t) { return __fadd_rn(a, t); }
};
template <> struct Tr<FLAME_BF16> {
    using T = uint16_t; using A = float; static constexpr int EPT = 8;
    __device__ static A ld(T x) { return bf16_to_f32(x); }
    __device__ static T st(A a) { return f32_to_bf16_exact(a); }
    __device__ static A tmp(T v, float r, double) { return bf16_round(__fmul_rn(bf16_to_f32(v), r)); }
    __device__ static A add(A a, A t) { return bf16_round(__fadd_rn(a, t)); }
};
template <> struct Tr<FLAME_F16> {
    using T = uint16_t; using A = float; static constexpr int EPT = 8;
    __device__ static A ld(T x) { return f16_to_f32(x); }
    __device__ static T st(A a) { return f32_to_f16_bits(a); }
    __device__ static A tmp(T v, float r, double) { return f16_round(__fmul_rn(f16_to_f32(v), r)); }
    __device__ static A add(A a, A t) { return f16_round(__fadd_rn(a, t)); }
};
template <> struct Tr<FLAME_F64> {
    using T = double; using A = double; static constexpr int EPT = 2;
    __device__ static A ld(T x) { return x; }
    __device__ static T st(A a) { return a; }
    __device__ static A tmp(T v, float, double r) { return __dmul_rn(v, r); }
    __device__ static A add(A a, A t) { return __dadd_rn(a, t); }
};
// int tensors: torch promotes int * python-float to fp32, then .to(int) truncates (fedavg.py:93-102)
template <> struct Tr<FLAME_I64> {
    using T = int64_t; using A = int64_t; static constexpr int EPT = 2;
    __device__ static A ld(T x) { return x; }
    __device__ static T st(A a) { return a; }
    __device__ static A tmp(T v, float r, double) { return static_cast<int64_t>(__fmul_rn(static_cast<float>(v), r)); }
    __device__ static A add(A a, A t) { return static_cast<int64_t>(static_cast<uint64_t>(a) + static_cast<uint64_t>(t)); }
};
template <> struct Tr<FLAME_I32> {
    using T = int32_t; using A = int32_t; static constexpr int EPT = 4;
    __device__ static A ld(T x) { return x; }
    __device__ static T st(A a) { return a; }
    __device__ static A tmp(T v, float r, double) { return static_cast<int32_t>(__fmul_rn(static_cast<float>(v), r)); }
    __device__ static A add(A a, A t) { return static_cast<int32_t>(static_cast<uint32_t>(a) + static_cast<uint32_t>(t)); }
};

template <int DT> constexpr int64_t chunk_elems() { return static_cast<int64_t>(kBlock) * kVPT * Tr<DT>::EPT; }

// ---------------------------------------------------------------- memory helpers
// All device data is accessed through address_space(1) (global) pointers so the
// compiler emits global_load/store (vmcnt only) instead of flat_* (which also
// count on lgkmcnt and would serialise against the scalar pointer/rate loads).
struct alignas(16) V16 { uint32_t w[4]; };
using u4 = __attribute__((ext_vector_type(4))) uint32_t;
template <typename T> using gptr = __attribute__((address_space(1))) T*;
template <typename T> using gcptr = const __attribute__((address_space(1))) T*;

template <typename T> __device__ __forceinline__ gcptr<T> G(const T* p) { return (gcptr<T>)(p); }
template <typename T> __device__ __forceinline__ gptr<T> G(T* p) { return (gptr<T>)(p); }

// Client updates are read exactly once: non-temporal loads.
__device__ __forceinline__ V16 ld_nt(const void* p) {
    u4 x = __builtin_nontemporal_load(G(reinterpret_cast<const u4*>(p)));
    V16 r; r.w[0] = x[0]; r.w[1] = x[1]; r.w[2] = x[2]; r.w[3] = x[3];
    return r;
}
__device__ __forceinline__ V16 ld_v(const void* p) {
    u4 x = *G(reinterpret_cast<const u4*>(p));
    V16 r; r.w[0] = x[0]; r.w[1] = x[1]; r.w[2] = x[2]; r.w[3] = x[3];
    return r;
}
// Output stores are write-through (sc0 sc1 nt): measured +2 % on config 3 and +4 % on
// 64-client bf16 against plain / nt stores, whose dirty L2 lines are written back
// interleaved with the client read stream (profiles/r01_scan5_*.log).  Inline asm
// because no builtin sets sc0/sc1; `s_nop 1` covers the store-data hazard.
__device__ __forceinline__ void st_v(void* p, const V16& v) {
    u4 x = {v.w[0], v.w[1], v.w[2], v.w[3]};
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt\n\ts_nop 1" :: "v"(p), "v"(x) : "memory");
}
// A plain (write-back) vector store: the slab insert, whose tiles are read again soon.
__device__ __forceinline__ void st_plain(void* p, const V16& v) {
    u4 x = {v.w[0], v.w[1], v.w[2], v.w[3]};
    *G(reinterpret_cast<u4*>(p)) = x;
}
template <typename T> __device__ __forceinline__ T ld1(const T* p) { return *G(p); }
template <typename T> __device__ __forceinline__ void st1(T* p, T x) { *G(p) = x; }
template <typename T, int EPT>
__device__ __forceinline__ void unpack(const V16& v, T (&x)[EPT]) {
    static_assert(sizeof(T) * EPT == 16, "lane vector is 16 bytes");
    __builtin_memcpy(x, v.w, 16);
}
template <typename T, int EPT>
__device__ __forceinline__ V16 pack(const T (&x)[EPT]) {
    V16 v;
    __builtin_memcpy(v.w, x, 16);
    return v;
}

// Wave-uniform segment lookup: largest s with segs[s].chunk_begin <= chunk.
template <typename SEG>
__device__ __forceinline__ int find_segment(const SEG* __restrict__ segs, int n_segs, int64_t chunk) {
    int lo = 0, hi = n_segs - 1;
    while (lo < hi) {
        int mid = (lo + hi + 1) >> 1;
        if (segs[mid].chunk_begin <= chunk) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// Byte offset of this lane's first element inside every client's data for the
// workgroup's chunk: contiguous (e0 * sizeof) or tiled (chunk * client_tile_stride + lane).
template <int DT, typename SEG>
__device__ __forceinline__ int64_t client_offset(const SEG& sg, int64_t chunk) {
    using T = typename Tr<DT>::T;
    const int64_t cl = chunk - sg.chunk_begin;
    const int64_t lane_elem = static_cast<int64_t>(threadIdx.x) * Tr<DT>::EPT;
    if (sg.client_tile_stride)
        return cl * sg.client_tile_stride + lane_elem * static_cast<int64_t>(sizeof(T));
    return (cl * chunk_elems<DT>() + lane_elem) * static_cast<int64_t>(sizeof(T));
}

// ---------------------------------------------------------------- reduction core
// A lane owns VPT 16-byte vectors of the chunk, at elements e0 + v*kBlock*EPT.
// Reduce clients [0, n) into acc for those slots.  VEC: every vector whole and
// aligned; else element-wise with bounds (tails / unaligned views).
template <int DT, int CU, bool VEC>
__device__ __forceinline__ void reduce_clients(typename Tr<DT>::A (&acc)[kVPT][Tr<DT>::EPT], bool init_first,
                                               const uint64_t* __restrict__ cp, int n,
                                               const float* __restrict__ r32, const double* __restrict__ r64,
                                               int64_t e0, int64_t numel, int64_t coff) {
    using X = Tr<DT>;
    using T = typename X::T;
    constexpr int EPT = X::EPT;
    constexpr int64_t VS = static_cast<int64_t>(kBlock) * EPT;  // vector stride in elements
    int i = 0;
    auto rate32 = [&](int c) -> float { if constexpr (DT == FLAME_F64) return 0.f; else return r32[c]; };
    auto rate64 = [&](int c) -> double { if constexpr (DT == FLAME_F64) return r64[c]; else return 0.0; };
    auto load_client = [&](int c, T (&x)[kVPT][EPT]) {
        const T* p = reinterpret_cast<const T*>(reinterpret_cast<const char*>(cp[c]) + coff);
#pragma unroll
        for (int v = 0; v < kVPT; ++v) {
            if constexpr (VEC) {
                unpack<T, EPT>(ld_nt(p + v * VS), x[v]);
            } else {
#pragma unroll
                for (int j = 0; j < EPT; ++j) x[v][j] = (e0 + v * VS + j < numel) ? ld1(p + v * VS + j) : T(0);
            }
        }
    };
    auto combine_r = [&](const float r, const double rd, const T (&x)[kVPT][EPT]) {
#pragma unroll
        for (int v = 0; v < kVPT; ++v)
#pragma unroll
            for (int j = 0; j < EPT; ++j) acc[v][j] = X::add(acc[v][j], X::tmp(x[v][j], r, rd));
    };
    auto combine = [&](int c, const T (&x)[kVPT][EPT]) { combine_r(rate32(c), rate64(c), x); };
    if (init_first && n > 0) {
        T x[kVPT][EPT];
        load_client(0, x);
        const float r = rate32(0);
        const double rd = rate64(0);
#pragma unroll
        for (int v = 0; v < kVPT; ++v)
#pragma unroll
            for (int j = 0; j < EPT; ++j) acc[v][j] = X::tmp(x[v][j], r, rd);
        i = 1;
    }
    for (; i + CU <= n; i += CU) {
        T x[CU][kVPT][EPT];
#pragma unroll
        for (int u = 0; u < CU; ++u) load_client(i + u, x[u]);
#pragma unroll
        for (int u = 0; u < CU; ++u) combine(i + u, x[u]);
    }
    for (; i < n; ++i) {
        T x[kVPT][EPT];
        load_client(i, x);
        combine(i, x);
    }
}

// One chunk of one segment: acc = base (or client 0), reduce every client in order.
// Full, aligned chunks hand their output vectors back (ov / op) so the caller can
// store them; tails and misaligned views store element-wise here.
template <int DT, int CU>
__device__ __forceinline__ bool reduce_chunk(const flame_segment* __restrict__ segs, int n_segs,
                                             const uint64_t* __restrict__ clients, int n_clients,
                                             const float* __restrict__ r32, const double* __restrict__ r64,
                                             unsigned flags, int64_t chunk, V16 (&ov)[kVPT],
                                             typename Tr<DT>::T*& op) {
    using X = Tr<DT>;
    using T = typename X::T;
    using A = typename X::A;
    constexpr int EPT = X::EPT;
    constexpr int64_t VS = static_cast<int64_t>(kBlock) * EPT;
    const int s = find_segment(segs, n_segs, chunk);
    const flame_segment sg = segs[s];
    const int64_t e0 = (chunk - sg.chunk_begin) * chunk_elems<DT>() + static_cast<int64_t>(threadIdx.x) * EPT;
    if (e0 >= sg.numel) return false;
    const uint64_t* cp = clients + static_cast<int64_t>(s) * n_clients;
    const int64_t coff = client_offset<DT>(sg, chunk);
    const bool init_first = (flags & FLAME_AGG_INIT_FIRST) != 0;
    if (flags & FLAME_AGG_SEG_RATES) {  // one rate row per segment
        if (r32) r32 += static_cast<int64_t>(s) * n_clients;
        if (r64) r64 += static_cast<int64_t>(s) * n_clients;
    }
    const bool vec = (e0 + (kVPT - 1) * VS + EPT <= sg.numel) && !(sg.flags & FLAME_SEG_UNALIGNED);
    A acc[kVPT][EPT];
    const T* bp = reinterpret_cast<const T*>(sg.in) + e0;
    op = reinterpret_cast<T*>(sg.out) + e0;
    if (vec) {
        if (!init_first) {
#pragma unroll
            for (int v = 0; v < kVPT; ++v) {
                T b[EPT];
                unpack<T, EPT>(ld_v(bp + v * VS), b);
#pragma unroll
                for (int j = 0; j < EPT; ++j) acc[v][j] = X::ld(b[j]);
            }
        }
        reduce_clients<DT, CU, true>(acc, init_first, cp, n_clients, r32, r64, e0, sg.numel, coff);
#pragma unroll
        for (int v = 0; v < kVPT; ++v) {
            T o[EPT];
#pragma unroll
            for (int j = 0; j < EPT; ++j) o[j] = X::st(acc[v][j]);
            ov[v] = pack<T, EPT>(o);
        }
        return true;
    }
    if (!init_first) {
#pragma unroll
        for (int v = 0; v < kVPT; ++v)
#pragma unroll
            for (int j = 0; j < EPT; ++j)
                acc[v][j] = X::ld((e0 + v * VS + j < sg.numel) ? ld1(bp + v * VS + j) : T(0));
    }
    reduce_clients<DT, 1, false>(acc, init_first, cp, n_clients, r32, r64, e0, sg.numel, coff);
#pragma unroll
    for (int v = 0; v < kVPT; ++v)
#pragma unroll
        for (int j = 0; j < EPT; ++j)
            if (e0 + v * VS + j < sg.numel) st1(op + v * VS + j, X::st(acc[v][j]));
    return false;
}

template <typename T>
__device__ __forceinline__ void store_chunk(T* op, const V16 (&ov)[kVPT]) {
    constexpr int64_t VS = static_cast<int64_t>(kBlock) * (16 / sizeof(T));
#pragma unroll
    for (int v = 0; v < kVPT; ++v) st_v(op + v * VS, ov[v]);
}

// Workgroup slot of block b when the 8 XCDs (dispatched round-robin) each take one
// contiguous eighth of the slots (FLAME_AGG_XCD_MAP / FLAME_OPT_XCD_MAP): a bijection.
__device__ __forceinline__ int64_t xcd_slot(int64_t b, int64_t n) {
    const int64_t q = n / 8, r = n % 8, x = b % 8;
    return x * q + (x < r ? x : r) + b / 8;
}

// G chunks per workgroup (G = 1: chunk = workgroup slot, in launch order or the XCD-contiguous
// map).  G > 1: the workgroup reduces chunks slot*G .. slot*G+G-1 one after another, holds their
// full output vectors in LDS and stores them in one burst at the end.
template <int DT, int CU, int G>
__device__ __forceinline__ void agg_reduce_body(const flame_segment* __restrict__ segs, int n_segs,
                                                const uint64_t* __restrict__ clients, int n_clients,
                                                const float* __restrict__ r32, const double* __restrict__ r64,
                                                unsigned flags, int64_t n_chunks) {
    using T = typename Tr<DT>::T;
    const int64_t slot = (flags & FLAME_AGG_XCD_MAP) ? xcd_slot(blockIdx.x, gridDim.x) : blockIdx.x;
    if constexpr (G == 1) {
        if (slot >= n_chunks) return;
        V16 ov[kVPT];
        T* op;
        if (reduce_chunk<DT, CU>(segs, n_segs, clients, n_clients, r32, r64, flags, slot, ov, op)) store_chunk(op, ov);
    } else {
        static_assert(G <= 32 && G * kVPT * kBlock * sizeof(V16) <= 128 * 1024, "agg_reduce_body: G chunks' outputs exceed the LDS");
        constexpr int64_t VS = static_cast<int64_t>(kBlock) * Tr<DT>::EPT;
        __shared__ V16 held[G * kVPT * kBlock];
        unsigned pending = 0;
#pragma unroll 1
        for (int g = 0; g < G; ++g) {
            const int64_t chunk = slot * G + g;
            if (chunk >= n_chunks) break;
            V16 ov[kVPT];
            T* op;
            if (reduce_chunk<DT, CU>(segs, n_segs, clients, n_clients, r32, r64, flags, chunk, ov, op)) {
#pragma unroll
                for (int v = 0; v < kVPT; ++v) held[(g * kVPT + v) * kBlock + threadIdx.x] = ov[v];
                pending |= 1u << g;
            }
        }
#pragma unroll 1
        for (int g = 0; g < G; ++g) {
            if (!(pending >> g & 1u)) continue;
            const int64_t chunk = slot * G + g;
            const flame_segment& sg = segs[find_segment(segs, n_segs, chunk)];
            T* op = reinterpret_cast<T*>(sg.out) + (chunk - sg.chunk_begin) * chunk_elems<DT>() +
                    static_cast<int64_t>(threadIdx.x) * Tr<DT>::EPT;
#pragma unroll
            for (int v = 0; v < kVPT; ++v) st_v(op + v * VS, held[(g * kVPT + v) * kBlock + threadIdx.x]);
        }
    }
}

template <int DT, int CU, int G>
__global__ __launch_bounds__(kBlock) void agg_reduce_kernel(const flame_segment* __restrict__ segs, int n_segs,
                                                            const uint64_t* __restrict__ clients, int n_clients,
                                                            const float* __restrict__ r32,
                                                            const double* __restrict__ r64, unsigned flags,
                                                            int64_t n_chunks) {
    agg_reduce_body<DT, CU, G>(segs, n_segs, clients, n_clients, r32, r64, flags, n_chunks);
}

// Small launches (few segments x few hundred clients): the whole metadata block travels as a
// kernel argument.  A separate H2D copy of a few KB is a blit kernel on gfx950 that the launch
// stream must run before the reduction (≈15 µs of GPU timeline per launch, measured on
// config 2: 0.171 -> 0.157 ms per step without it); kernel arguments reach the GPU with the
// dispatch itself and are read through the scalar cache like the device-resident table.
constexpr int kArgMetaWords = 448;          // 3,584 B: kernel arguments are limited to 4 KiB
struct ArgMeta { uint64_t w[kArgMetaWords]; };

template <int DT, int CU, int G>
__global__ __launch_bounds__(kBlock) void agg_reduce_kernel_argmeta(const ArgMeta meta, int n_segs, int n_clients,
                                                                    int off_clients, int off_r32, int off_r64,
                                                                    unsigned flags, int64_t n_chunks) {
    // `meta` is the first kernel argument: read it in place in the kernarg segment (scalar
    // loads) -- naming the by-value parameter would copy 3.5 KB into every lane's scratch
    (void)sizeof(meta);
    const uint64_t* w = (const uint64_t*)__builtin_amdgcn_kernarg_segment_ptr();
    agg_reduce_body<DT, CU, G>(reinterpret_cast<const flame_segment*>(w), n_segs, w + off_clients, n_clients,
                            off_r32 >= 0 ? reinterpret_cast<const float*>(w + off_r32) : nullptr,
                            off_r64 >= 0 ? reinterpret_cast<const double*>(w + off_r64) : nullptr, flags, n_chunks);
}

// ---------------------------------------------------------------- fused FedOPT (fp32)
__device__ __forceinline__ float sign_f(float x) {  // torch.sign: NaN -> 0, -0 -> 0
    if constexpr (kYogiSelect) {
        // +-1 with x's sign where x is ordered and nonzero (one v_cmp_lg_f32 + one v_bfi_b32),
        // else +0: the same value as the integer difference below, in 3 instructions instead of 6
        return __builtin_islessgreater(x, 0.0f) ? __builtin_copysignf(1.0f, x) : 0.0f;
    } else {
        return static_cast<float>((0.0f < x) - (x < 0.0f));
    }
}

// Per-dtype rounding after each reference op (identity for fp32; RNE to bf16 / fp16).
template <int DT> __device__ __forceinline__ float rnd(float x) {
    if constexpr (DT == FLAME_BF16) return bf16_round(x);
    else if constexpr (DT == FLAME_F16) return f16_round(x);
    else return x;
}

// fedopt.py:106-129 (+ the _delta_v variants) up to the square root: d, the new m and v, and
// the numerator eta * m, each torch op rounded in the tensor's dtype.
template <int DT, int VARIANT>
__device__ __forceinline__ void adapt_moments(float avg, float cur, float& m, float& v, float& num, float b1,
                                              float omb1, float b2, float omb2, float eta) {
    const float d = rnd<DT>(__fsub_rn(avg, cur));
    const float mn = rnd<DT>(__fadd_rn(rnd<DT>(__fmul_rn(b1, m)), rnd<DT>(__fmul_rn(omb1, d))));
    const float d2 = rnd<DT>(__fmul_rn(d, d));
    float vn;
    if constexpr (VARIANT == FLAME_FEDADAM) {
        vn = rnd<DT>(__fadd_rn(rnd<DT>(__fmul_rn(b2, v)), rnd<DT>(__fmul_rn(omb2, d2))));
    } else if constexpr (VARIANT == FLAME_FEDYOGI) {
        const float t = rnd<DT>(__fmul_rn(omb2, d2));
        vn = rnd<DT>(__fsub_rn(v, rnd<DT>(__fmul_rn(t, sign_f(rnd<DT>(__fsub_rn(v, d2)))))));
    } else {
        vn = rnd<DT>(__fadd_rn(v, d2));
    }
    m = mn;
    v = vn;
    num = rnd<DT>(__fmul_rn(eta, mn));
}

// One element of fedopt.py:106-129, each torch op rounded in the tensor's dtype.  `tau` arrives
// pre-rounded to the dtype for bf16/fp16 (torch-CPU rounds a Python scalar to a reduced-precision
// tensor's dtype before + and -, not before * and /).  The general correctly rounded sqrt and
// divide (__builtin_sqrtf is correctly rounded; the __fsqrt_rn builtin lowers to the 1-ulp
// v_sqrt_f32): the scalar tail path, and adapt_vec's fallback.
template <int DT, int VARIANT>
__device__ __forceinline__ void adapt_elem(float avg, float cur, float& m, float& v, float& cur_out,
                                           float b1, float omb1, float b2, float omb2, float eta, float tau) {
    float num;
    adapt_moments<DT, VARIANT>(avg, cur, m, v, num, b1, omb1, b2, omb2, eta);
    const float den = rnd<DT>(__fadd_rn(rnd<DT>(__builtin_sqrtf(v)), tau));
    cur_out = rnd<DT>(__fadd_rn(cur, rnd<DT>(__fdiv_rn(num, den))));
}

// A lane's EPT elements of one adaptive step (cur_is_avg: current IS the average, d = 0).  When
// the lane's operands are all in the range fastmath.h admits -- v in [+0, 2^78], eta*m = +-0 or
// 2^-85 <= |.| <= 2^100, tau in [2^-20, 2^38] (so sqrt(v) + tau is in [2^-20, 2^40]) -- the
// square root and the divide take flame_fm::sqrt_rn / div_rn (rsq / rcp seeds, packed fma), else
// the general sequences.  Both give the same m, v and current (tools/fp_probe.py), so which one a
// lane takes never shows in the results.
// bf16 (a lane's 8 elements as 4 pairs): adapt_vec's op sequence with every fp32 op on a pair
// (v_pk_mul_f32 / v_pk_add_f32) and every bf16 rounding one instruction (bf16_rnd1).  Admitted
// lanes take v_sqrt_f32 and num * v_rcp_f32(den) for the correctly rounded root and quotient: both
// are within 2 fp32 ulps of the exact value, and the exact root of a bf16 v, and the exact quotient
// of two bf16 values, are never within 2^-18 (relative) of a bf16 rounding midpoint (8-bit
// significands), so the bf16 rounding of either equals the bf16 rounding of the correctly rounded
// fp32 value (v_sqrt_f32 flushes a subnormal v to a zero root, but den = RN(RN(root) + tau) = tau
// for both roots there).  tools/fp_probe.py checks the root on every normal bf16 v, den on every
// admitted v and the quotient on every admitted (num, den) pair.
// fp16: the same sequence with f16_rnd2 (one v_cvt_pk_f16_f32 + two widening converts per pair).
// An fp16 significand has 11 bits, too many for the midpoint argument; the exhaustive fp16 probe
// of tools/fp_probe.py finds v_sqrt_f32 exact under the fp16 rounding on every finite v (so the
// root takes it, FLAME_T_F16_HWROOT) but num * v_rcp_f32 not (the quotient stays div_rn).
// The pair rounding (inline asm: never on a transcendental's result) and the single rounding the
// compiler builds (safe on one) of the 16-bit dtypes.
template <int DT> __device__ __forceinline__ f2 hrnd2(f2 x) {
    if constexpr (DT == FLAME_BF16) return bf16_rnd2(x);
    else return f16_rnd2(x);
}
template <int DT> __device__ __forceinline__ float hrnd1(float x) {
    if constexpr (DT == FLAME_BF16) return bf16_round(x);
    else return f16_round(x);
}

template <int DT, int VARIANT>
__device__ __forceinline__ void adapt_vec_half(const float (&avg)[8], const float (&cur)[8], bool cur_is_avg,
                                               float (&m)[8], float (&v)[8], float (&cur_out)[8], float b1,
                                               float omb1, float b2, float omb2, float eta, float tau) {
    float c[8], num[8];
#pragma unroll
    for (int p = 0; p < 8; p += 2) {
        const f2 a = {avg[p], avg[p + 1]};
        const f2 cc = cur_is_avg ? a : f2{cur[p], cur[p + 1]};
        const f2 d = hrnd2<DT>(a - cc);
        const f2 mn = hrnd2<DT>(hrnd2<DT>(splat2(b1) * f2{m[p], m[p + 1]}) + hrnd2<DT>(splat2(omb1) * d));
        const f2 d2 = hrnd2<DT>(d * d);
        const f2 vo = {v[p], v[p + 1]};
        f2 vn;
        if constexpr (VARIANT == FLAME_FEDADAM) {
            vn = hrnd2<DT>(hrnd2<DT>(splat2(b2) * vo) + hrnd2<DT>(splat2(omb2) * d2));
        } else if constexpr (VARIANT == FLAME_FEDYOGI) {
            const f2 t = hrnd2<DT>(splat2(omb2) * d2);
            const f2 x = hrnd2<DT>(vo - d2);
            // t * sign(x) needs no rounding of its own: t is in the dtype and the sign +-1 or +0, so
            // the product is +-t or +-0 exactly (a NaN stays a NaN; its payload bits are not pinned)
            vn = hrnd2<DT>(vo - t * f2{sign_f(x.x), sign_f(x.y)});
        } else {
            vn = hrnd2<DT>(vo + d2);
        }
        const f2 nm = hrnd2<DT>(splat2(eta) * mn);
        c[p] = cc.x;
        c[p + 1] = cc.y;
        m[p] = mn.x;
        m[p + 1] = mn.y;
        v[p] = vn.x;
        v[p + 1] = vn.y;
        num[p] = nm.x;
        num[p + 1] = nm.y;
    }
    bool adm;
    if constexpr (!kHalfAdmit) adm = flame_fm::admits<8>(v, num);
    else if constexpr (DT == FLAME_BF16) adm = flame_fm::admits_v<8>(v);
    else adm = flame_fm::admits_v<8>(v) & flame_fm::admits_finite<8>(num) & (tau <= 0x1p15f);  // den finite in fp16
    const bool ok = (tau >= 0x1p-20f) & (tau <= 0x1p38f) & adm;
    if (ok) {
        constexpr bool hw_root = DT == FLAME_BF16 || kF16HwRoot;
        constexpr bool hw_div = DT == FLAME_BF16;
#pragma unroll
        for (int p = 0; p < 8; p += 2) {
            // the roots' rounding through hrnd1: a v_sqrt_f32 / v_rsq_f32 result never feeds inline asm
            f2 s, q;
            if constexpr (hw_root) {
                s = f2{hrnd1<DT>(__builtin_amdgcn_sqrtf(v[p])), hrnd1<DT>(__builtin_amdgcn_sqrtf(v[p + 1]))};
            } else {
                s = f2{hrnd1<DT>(flame_fm::sqrt_rn(v[p])), hrnd1<DT>(flame_fm::sqrt_rn(v[p + 1]))};
            }
            const f2 den = hrnd2<DT>(s + splat2(tau));
            if constexpr (hw_div) {
                q = hrnd2<DT>(f2{num[p], num[p + 1]} * f2{__builtin_amdgcn_rcpf(den.x), __builtin_amdgcn_rcpf(den.y)});
            } else {
                q = hrnd2<DT>(f2{flame_fm::div_rn(num[p], den.x), flame_fm::div_rn(num[p + 1], den.y)});
            }
            const f2 co = hrnd2<DT>(f2{c[p], c[p + 1]} + q);
            cur_out[p] = co.x;
            cur_out[p + 1] = co.y;
        }
    } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float den = hrnd1<DT>(__fadd_rn(hrnd1<DT>(__builtin_sqrtf(v[j])), tau));
            cur_out[j] = hrnd1<DT>(__fadd_rn(c[j], hrnd1<DT>(__fdiv_rn(num[j], den))));
        }
    }
}

template <int DT, int VARIANT, int EPT>
__device__ __forceinline__ void adapt_vec(const float (&avg)[EPT], const float (&cur)[EPT], bool cur_is_avg,
                                          float (&m)[EPT], float (&v)[EPT], float (&cur_out)[EPT], float b1,
                                          float omb1, float b2, float omb2, float eta, float tau) {
    if constexpr (EPT == 8 && ((DT == FLAME_BF16 && kBf16Packed) || (DT == FLAME_F16 && kF16Packed))) {
        adapt_vec_half<DT, VARIANT>(avg, cur, cur_is_avg, m, v, cur_out, b1, omb1, b2, omb2, eta, tau);
        return;
    }
    float c[EPT], num[EPT];
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
        c[j] = cur_is_avg ? avg[j] : cur[j];
        adapt_moments<DT, VARIANT>(avg[j], c[j], m[j], v[j], num[j], b1, omb1, b2, omb2, eta);
    }
    const bool ok = (tau >= 0x1p-20f) & (tau <= 0x1p38f) & flame_fm::admits<EPT>(v, num);
    if (ok) {         // per lane (exec-masked; a wave whose lanes all agree runs one side only)
#pragma unroll
        for (int j = 0; j < EPT; ++j) {
            const float den = rnd<DT>(__fadd_rn(rnd<DT>(flame_fm::sqrt_rn(v[j])), tau));
            cur_out[j] = rnd<DT>(__fadd_rn(c[j], rnd<DT>(flame_fm::div_rn(num[j], den))));
        }
    } else {
#pragma unroll
        for (int j = 0; j < EPT; ++j) {
            const float den = rnd<DT>(__fadd_rn(rnd<DT>(__builtin_sqrtf(v[j])), tau));
            cur_out[j] = rnd<DT>(__fadd_rn(c[j], rnd<DT>(__fdiv_rn(num[j], den))));
        }
    }
}

// One chunk of a FedOPT round.  held != nullptr: a full-vector chunk leaves its avg / m / v /
// cur blocks in LDS (held[(o * kVPT + v) * kBlock + lane], o = avg, m, v, cur) for the caller
// to store, and returns true; otherwise everything is stored here and it returns false.
template <int DT, int VARIANT, int CU>
__device__ __forceinline__ bool fedopt_chunk(const flame_segment* __restrict__ segs, int n_segs, int64_t chunk,
                                             const uint64_t* __restrict__ clients, int n_clients,
                                             const float* __restrict__ r32, unsigned flags, float b1,
                                             float omb1, float b2, float omb2, float eta, float tau,
                                             V16* held) {
    using X = Tr<DT>;
    using T = typename X::T;
    constexpr int EPT = X::EPT;
    constexpr int64_t VS = static_cast<int64_t>(kBlock) * EPT;
    const int s = find_segment(segs, n_segs, chunk);
    const flame_segment sg = segs[s];
    const int64_t e0 = (chunk - sg.chunk_begin) * chunk_elems<DT>() + static_cast<int64_t>(threadIdx.x) * EPT;
    if (e0 >= sg.numel) return false;
    const uint64_t* cp = clients + static_cast<int64_t>(s) * n_clients;
    const int64_t coff = client_offset<DT>(sg, chunk);
    const bool zero_state = (flags & FLAME_OPT_STATE_ZERO) != 0;
    const bool cur_avg = (sg.flags & FLAME_SEG_CUR_IS_AVG) != 0;   // cur IS the FedAvg result
    const bool vec = (e0 + (kVPT - 1) * VS + EPT <= sg.numel) && !(sg.flags & FLAME_SEG_UNALIGNED);
    float acc[kVPT][EPT];
    const T* base = reinterpret_cast<const T*>(sg.in) + e0;
    const T* curp = reinterpret_cast<const T*>(sg.cur) + e0;
    T* mp = reinterpret_cast<T*>(sg.m) + e0;
    T* vp = reinterpret_cast<T*>(sg.v) + e0;
    T* ap = sg.out ? reinterpret_cast<T*>(sg.out) + e0 : nullptr;
    T* cop = reinterpret_cast<T*>(sg.cur_out) + e0;
    if (vec) {
#pragma unroll
        for (int v = 0; v < kVPT; ++v) {
            T b[EPT];
            unpack<T, EPT>(ld_v(base + v * VS), b);
#pragma unroll
            for (int j = 0; j < EPT; ++j) acc[v][j] = X::ld(b[j]);
        }
        reduce_clients<DT, CU, true>(acc, false, cp, n_clients, r32, nullptr, e0, sg.numel, coff);
#pragma unroll
        for (int v = 0; v < kVPT; ++v) {
            T cur_t[EPT], m_t[EPT], v_t[EPT], avg_o[EPT], m_o[EPT], v_o[EPT], c_o[EPT];
            if (!cur_avg) unpack<T, EPT>(ld_v(curp + v * VS), cur_t);
            if (!zero_state) {
                unpack<T, EPT>(ld_v(mp + v * VS), m_t);
                unpack<T, EPT>(ld_v(vp + v * VS), v_t);
            }
            float cf[EPT], mf[EPT], vf[EPT], co[EPT];
#pragma unroll
            for (int j = 0; j < EPT; ++j) {
                cf[j] = cur_avg ? 0.f : X::ld(cur_t[j]);
                mf[j] = zero_state ? 0.f : X::ld(m_t[j]);
                vf[j] = zero_state ? 0.f : X::ld(v_t[j]);
            }
            adapt_vec<DT, VARIANT, EPT>(acc[v], cf, cur_avg, mf, vf, co, b1, omb1, b2, omb2, eta, tau);
#pragma unroll
            for (int j = 0; j < EPT; ++j) {
                avg_o[j] = X::st(acc[v][j]);
                m_o[j] = X::st(mf[j]);
                v_o[j] = X::st(vf[j]);
                c_o[j] = X::st(co[j]);
            }
            if (held) {
                V16* h = held + v * kBlock + threadIdx.x;
                h[0 * kVPT * kBlock] = pack<T, EPT>(avg_o);
                h[1 * kVPT * kBlock] = pack<T, EPT>(m_o);
                h[2 * kVPT * kBlock] = pack<T, EPT>(v_o);
                h[3 * kVPT * kBlock] = pack<T, EPT>(c_o);
                continue;
            }
            if (ap) st_v(ap + v * VS, pack<T, EPT>(avg_o));
            st_v(mp + v * VS, pack<T, EPT>(m_o));
            st_v(vp + v * VS, pack<T, EPT>(v_o));
            st_v(cop + v * VS, pack<T, EPT>(c_o));
        }
        return held != nullptr;
    } else {
#pragma unroll
        for (int v = 0; v < kVPT; ++v)
#pragma unroll
            for (int j = 0; j < EPT; ++j)
                acc[v][j] = (e0 + v * VS + j < sg.numel) ? X::ld(ld1(base + v * VS + j)) : 0.f;
        reduce_clients<DT, 1, false>(acc, false, cp, n_clients, r32, nullptr, e0, sg.numel, coff);
#pragma unroll
        for (int v = 0; v < kVPT; ++v)
#pragma unroll
            for (int j = 0; j < EPT; ++j) {
                const int64_t o = v * VS + j;
                if (e0 + o >= sg.numel) continue;
                float mj = zero_state ? 0.f : X::ld(ld1(mp + o)), vj = zero_state ? 0.f : X::ld(ld1(vp + o)), cj;
                adapt_elem<DT, VARIANT>(acc[v][j], cur_avg ? acc[v][j] : X::ld(ld1(curp + o)), mj, vj, cj, b1, omb1,
                                        b2, omb2, eta, tau);
                if (ap) st1(ap + o, X::st(acc[v][j]));
                st1(mp + o, X::st(mj));
                st1(vp + o, X::st(vj));
                st1(cop + o, X::st(cj));
            }
    }
    return false;
}

// G = 1: one chunk per workgroup, stored as computed.  G > 1: G consecutive chunks per
// workgroup, their outputs held in LDS and stored together at the end (kOptWGC).
template <int DT, int VARIANT, int CU, int G>
__device__ __forceinline__ void fedopt_body(const flame_segment* __restrict__ segs, int n_segs,
                                            const uint64_t* __restrict__ clients, int n_clients,
                                            const float* __restrict__ r32, unsigned flags, float b1,
                                            float omb1, float b2, float omb2, float eta, float tau,
                                            int64_t n_chunks) {
    const int64_t wg = (flags & FLAME_OPT_XCD_MAP) ? xcd_slot(blockIdx.x, gridDim.x) : blockIdx.x;
    if constexpr (G == 1) {
        (void)n_chunks;
        fedopt_chunk<DT, VARIANT, CU>(segs, n_segs, wg, clients, n_clients, r32, flags, b1, omb1, b2,
                                      omb2, eta, tau, nullptr);
    } else {
        using T = typename Tr<DT>::T;
        constexpr int64_t VS = static_cast<int64_t>(kBlock) * Tr<DT>::EPT;
        static_assert(G * 4 * kVPT * kBlock * sizeof(V16) <= 160 * 1024, "kOptWGC: outputs exceed the LDS");
        __shared__ V16 held[G * 4 * kVPT * kBlock];
        unsigned pending = 0;
#pragma unroll 1
        for (int g = 0; g < G; ++g) {
            const int64_t chunk = wg * G + g;
            if (chunk >= n_chunks) break;
            if (fedopt_chunk<DT, VARIANT, CU>(segs, n_segs, chunk, clients, n_clients, r32, flags, b1, omb1, b2, omb2,
                                              eta, tau, held + g * 4 * kVPT * kBlock))
                pending |= 1u << g;
        }
#pragma unroll 1
        for (int g = 0; g < G; ++g) {
            if (!(pending >> g & 1u)) continue;
            const int64_t chunk = wg * G + g;
            const flame_segment& sg = segs[find_segment(segs, n_segs, chunk)];
            const int64_t e0 = (chunk - sg.chunk_begin) * chunk_elems<DT>() +
                               static_cast<int64_t>(threadIdx.x) * Tr<DT>::EPT;
            T* outs[4] = {sg.out ? reinterpret_cast<T*>(sg.out) + e0 : nullptr, reinterpret_cast<T*>(sg.m) + e0,
                          reinterpret_cast<T*>(sg.v) + e0, reinterpret_cast<T*>(sg.cur_out) + e0};
#pragma unroll
            for (int o = 0; o < 4; ++o) {
                if (!outs[o]) continue;
#pragma unroll
                for (int v = 0; v < kVPT; ++v)
                    st_v(outs[o] + v * VS, held[((g * 4 + o) * kVPT + v) * kBlock + threadIdx.x]);
            }
        }
    }
}

template <int DT, int VARIANT, int CU, int G>
__global__ __launch_bounds__(kBlock) void fedopt_kernel(const flame_segment* __restrict__ segs, int n_segs,
                                                        const uint64_t* __restrict__ clients, int n_clients,
                                                        const float* __restrict__ r32, unsigned flags, float b1,
                                                        float omb1, float b2, float omb2, float eta, float tau,
                                                        int64_t n_chunks) {
    fedopt_body<DT, VARIANT, CU, G>(segs, n_segs, clients, n_clients, r32, flags, b1, omb1, b2, omb2, eta, tau,
                                    n_chunks);
}

// The same with the metadata block as a kernel argument, read in place (flame_fedopt_reduce_adapt_argmeta;
// see agg_reduce_kernel_argmeta).  Word offsets: client table at off_clients, fp32 rates at off_r32.
template <int DT, int VARIANT, int CU, int G>
__global__ __launch_bounds__(kBlock) void fedopt_kernel_argmeta(const ArgMeta meta, int n_segs, int n_clients,
                                                                int off_clients, int off_r32, unsigned flags,
                                                                float b1, float omb1, float b2, float omb2,
                                                                float eta, float tau, int64_t n_chunks) {
    (void)sizeof(meta);
    const uint64_t* w = (const uint64_t*)__builtin_amdgcn_kernarg_segment_ptr();
    fedopt_body<DT, VARIANT, CU, G>(reinterpret_cast<const flame_segment*>(w), n_segs, w + off_clients, n_clients,
                                    off_r32 >= 0 ? reinterpret_cast<const float*>(w + off_r32) : nullptr, flags,
                                    b1, omb1, b2, omb2, eta, tau, n_chunks);
}

// ---------------------------------------------------------------- eager FedOPT chain
// The eager top aggregator's round (eager_syncfl/top_aggregator.py:36-90) calls do() once per
// arrival: FedAvg of that arrival into the round's base (fedavg.py:93-104), then one adaptive
// step from the optimizer's state (fedopt.py:102-129).  This kernel runs a queue of such calls in
// one pass.  Per element, for each client i in arrival order:
//   b = b + tmp(w_i, r_i)
//   where client i closes a do() call (step_end[i] != 0): d = b - c, m / v / c updated as
//   adapt_elem (c = b for the first step when the segment is flagged FLAME_SEG_CUR_IS_AVG:
//   current_weights IS the base right after the round-1 passthrough).
// Base, current, m and v are read once and base, m, v and the new current written once, instead
// of every arrival's launch reading and writing all four.  Bitwise equal to those launches: every
// value held in registers between steps is already rounded to the dtype (each op rounds), so it
// equals what the per-arrival launches store and reload.
// step_end[i] through a SCALAR load: the aligned dword holding byte i (never outside the page
// that holds it), so the per-step test is an s_load + scalar branch, not a vector byte load whose
// s_waitcnt vmcnt(0) would also wait for the batch's client loads in flight.
__device__ __forceinline__ bool step_ends(const uint8_t* __restrict__ step_end, int i) {
    using kptr = const __attribute__((address_space(4))) uint32_t*;    // constant: scalar loads
    const uintptr_t a = reinterpret_cast<uintptr_t>(step_end) + static_cast<uintptr_t>(i);
    const uint32_t w = *reinterpret_cast<kptr>(a & ~static_cast<uintptr_t>(3));
    return ((w >> ((a & 3u) * 8u)) & 0xffu) != 0u;
}

// VEC: the workgroup's whole chunk is inside the segment and aligned, so every lane's loads are
// unconditional 16-byte vectors and the batch's loads are waited for one by one
// (s_waitcnt vmcnt(CU - 1 - u)) instead of all at once.
template <int DT, int VARIANT, int CU, bool VEC>
__device__ __forceinline__ void fedopt_chain_body(const flame_segment& sg, int64_t e0, const uint64_t* __restrict__ cp,
                                                  int64_t coff, int n_clients, const float* __restrict__ r32,
                                                  const uint8_t* __restrict__ step_end, unsigned flags, float b1,
                                                  float omb1, float b2, float omb2, float eta, float tau) {
    using X = Tr<DT>;
    using T = typename X::T;
    constexpr int EPT = X::EPT;
    const int nv = VEC ? EPT : static_cast<int>(sg.numel - e0 < EPT ? sg.numel - e0 : EPT);
    bool aliased = (sg.flags & FLAME_SEG_CUR_IS_AVG) != 0;
    const bool zero_state = (flags & FLAME_OPT_STATE_ZERO) != 0;
    const T* bp = reinterpret_cast<const T*>(sg.in) + e0;
    const T* curp = reinterpret_cast<const T*>(sg.cur) + e0;
    T* mp = reinterpret_cast<T*>(sg.m) + e0;
    T* vp = reinterpret_cast<T*>(sg.v) + e0;
    auto load_t = [&](const T* p, T (&x)[EPT], bool nt) {
        if constexpr (VEC) {
            unpack<T, EPT>(nt ? ld_nt(p) : ld_v(p), x);
        } else {
#pragma unroll
            for (int j = 0; j < EPT; ++j) x[j] = j < nv ? ld1(p + j) : T(0);
        }
    };
    auto load_f = [&](const T* p, float (&x)[EPT]) {
        T t[EPT];
        load_t(p, t, false);
#pragma unroll
        for (int j = 0; j < EPT; ++j) x[j] = X::ld(t[j]);
    };
    float b[EPT], c[EPT] = {}, m[EPT], v[EPT];
    load_f(bp, b);
    if (!aliased) load_f(curp, c);
    if (zero_state) {
#pragma unroll
        for (int j = 0; j < EPT; ++j) m[j] = v[j] = 0.f;
    } else {
        load_f(mp, m);
        load_f(vp, v);
    }
    auto load_client = [&](int i, T (&x)[EPT]) {
        load_t(reinterpret_cast<const T*>(reinterpret_cast<const char*>(cp[i]) + coff), x, true);
    };
    auto arrive = [&](const T (&x)[EPT], float r, bool ends) {
        if constexpr ((DT == FLAME_BF16 && kBf16Packed) || (DT == FLAME_F16 && kF16Packed)) {
#pragma unroll
            for (int j = 0; j < EPT; j += 2) {     // X::add(b, X::tmp(x, r)) on pairs
                const f2 t = hrnd2<DT>(f2{X::ld(x[j]), X::ld(x[j + 1])} * splat2(r));
                const f2 s = hrnd2<DT>(f2{b[j], b[j + 1]} + t);
                b[j] = s.x;
                b[j + 1] = s.y;
            }
        } else {
#pragma unroll
            for (int j = 0; j < EPT; ++j) b[j] = X::add(b[j], X::tmp(x[j], r, 0.0));
        }
        if (ends) {     // uniform: one do() call ends here
            if (__builtin_expect(aliased, 0)) {   // the first step after the passthrough: current IS base
#pragma unroll
                for (int j = 0; j < EPT; ++j) c[j] = b[j];
                aliased = false;
            }
            adapt_vec<DT, VARIANT, EPT>(b, c, false, m, v, c, b1, omb1, b2, omb2, eta, tau);
        }
    };
    auto load_batch = [&](int i0, T (&x)[CU][EPT], float (&rr)[CU], bool (&ends)[CU]) {
#pragma unroll
        for (int u = 0; u < CU; ++u) load_client(i0 + u, x[u]);
#pragma unroll
        for (int u = 0; u < CU; ++u) {     // the batch's scalar loads issued together, one wait
            rr[u] = r32[i0 + u];
            ends[u] = step_ends(step_end, i0 + u);
        }
    };
    auto run_batch = [&](const T (&x)[CU][EPT], const float (&rr)[CU], const bool (&ends)[CU]) {
#pragma unroll
        for (int u = 0; u < CU; ++u) arrive(x[u], rr[u], ends[u]);
    };
    int i = 0;
    // (Two register batches -- the next batch's loads issued before this one's steps -- run no
    // faster: 1.294 vs 1.287 ms at 8 loads per batch, 1.457 at 12, 3.40 at 16 (two 64-register
    // batches); one process, bitwise, profiles/r05k_chain_pipe_ab.log.  Nor do two or four
    // chunks per lane -- twice / four times the independent step chains: 1.38-1.44 vs 1.378 ms,
    // profiles/r05o_chain_ev_ab.log -- nor 2 / 3 / 4 chunks per workgroup with their outputs burst
    // from LDS: 1.386 / 1.417 / 1.372 vs 1.370 ms, profiles/r05w_chain_wgc_ab.log.  Three resident
    // workgroups of the plain batch loop already overlap one another's loads and arithmetic.)
    for (; i + CU <= n_clients; i += CU) {
        T x[CU][EPT];
        float rr[CU];
        bool ends[CU];
        load_batch(i, x, rr, ends);
        run_batch(x, rr, ends);
    }
    for (; i < n_clients; ++i) {
        T x[EPT];
        load_client(i, x);
        arrive(x, r32[i], step_ends(step_end, i));
    }
    if (aliased) {             // no step closed: current is still the base
#pragma unroll
        for (int j = 0; j < EPT; ++j) c[j] = b[j];
    }
    T* outs[4] = {reinterpret_cast<T*>(sg.out) + e0, mp, vp, reinterpret_cast<T*>(sg.cur_out) + e0};
    const float* vals[4] = {b, m, v, c};
#pragma unroll
    for (int o = 0; o < 4; ++o) {
        T t[EPT];
#pragma unroll
        for (int j = 0; j < EPT; ++j) t[j] = X::st(vals[o][j]);
        if constexpr (VEC) {
            st_v(outs[o], pack<T, EPT>(t));
        } else {
            for (int j = 0; j < nv; ++j) st1(outs[o] + j, t[j]);
        }
    }
}

// fedopt_chain_body for an fp16 model on a full, aligned chunk: the same per-arrival accumulate and
// per-call step (fedopt.py:102-129, each torch op rounded to fp16), with the lane's 8 elements held
// as 4 packed pairs.  An op whose operands are both fp16 is one packed fp16 instruction (same bits
// as fp32-then-fp16, see h2 above); a product with a Python scalar is smul_h2; the root and the
// quotient widen their operands and take v_sqrt_f32 / flame_fm::div_rn as adapt_vec_half does
// (same admission: v in [+0, 65504] per half, a finite numerator, tau in [2^-20, 2^15]); a lane
// outside it takes the general sequence per element.
template <int VARIANT, int CU>
__device__ __forceinline__ void fedopt_chain_body_f16(const flame_segment& sg, int64_t e0, const uint64_t* __restrict__ cp,
                                                      int64_t coff, int n_clients, const float* __restrict__ r32,
                                                      const uint8_t* __restrict__ step_end, unsigned flags, float b1,
                                                      float omb1, float b2, float omb2, float eta, float tau) {
    bool aliased = (sg.flags & FLAME_SEG_CUR_IS_AVG) != 0;
    const bool zero_state = (flags & FLAME_OPT_STATE_ZERO) != 0;
    const uint16_t* bp = reinterpret_cast<const uint16_t*>(sg.in) + e0;
    const uint16_t* curp = reinterpret_cast<const uint16_t*>(sg.cur) + e0;
    uint16_t* mp = reinterpret_cast<uint16_t*>(sg.m) + e0;
    uint16_t* vp = reinterpret_cast<uint16_t*>(sg.v) + e0;
    uint32_t b[4], c[4] = {}, m[4] = {}, v[4] = {};
    auto ld4 = [](const void* p, uint32_t (&x)[4]) {
        const V16 t = ld_v(p);
#pragma unroll
        for (int q = 0; q < 4; ++q) x[q] = t.w[q];
    };
    ld4(bp, b);
    if (!aliased) ld4(curp, c);
    if (!zero_state) {
        ld4(mp, m);
        ld4(vp, v);
    }
    const h2 tau2 = {static_cast<_Float16>(tau), static_cast<_Float16>(tau)};   // tau is fp16-exact
    const bool tau_ok = (tau >= 0x1p-20f) & (tau <= 0x1p15f);                   // den in [2^-20, 65504]
    auto adapt = [&]() {
        uint32_t num[4];
        us2 vmax = {0, 0};
        bool fin = true;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const h2 d = h2_of(b[p]) - h2_of(c[p]);
            const h2 mn = h2_of(smul_h2(b1, m[p])) + h2_of(smul_h2(omb1, u_of(d)));
            const h2 d2 = d * d;
            const h2 vo = h2_of(v[p]);
            h2 vn;
            if constexpr (VARIANT == FLAME_FEDADAM) {
                vn = h2_of(smul_h2(b2, v[p])) + h2_of(smul_h2(omb2, u_of(d2)));
            } else if constexpr (VARIANT == FLAME_FEDYOGI) {
                const h2 t = h2_of(smul_h2(omb2, u_of(d2)));
                vn = vo - t * sign_h2(vo - d2);      // t * (+-1 or +0) is exact
            } else {
                vn = vo + d2;
            }
            m[p] = u_of(mn);
            v[p] = u_of(vn);
            float plo, phi;
            num[p] = smul_h2(eta, m[p], plo, phi);
            vmax = __builtin_elementwise_max(vmax, __builtin_bit_cast(us2, v[p]));
            // compares (lane masks), not fmaxf: an fmaxf of an inline-asm result costs a
            // canonicalizing max first
            fin &= (__builtin_fabsf(plo) < 65520.f) & (__builtin_fabsf(phi) < 65520.f);
        }
        // v's halves in [+0, 65504] (a sign, an inf or a NaN is above 0x7bff); every numerator
        // finite: its fp32 product below 65520, the fp16 overflow threshold (a NaN product fails the
        // compare: that lane takes the general sequence, which gives the same NaN)
        const bool ok = tau_ok & (max(vmax.x, vmax.y) <= 0x7bffu) & fin;
        if (ok) {
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                h2 s;
                if constexpr (kF16HalfRoot) {
                    s = __builtin_elementwise_sqrt(h2_of(v[p]));      // v_sqrt_f16 (tools/fp_probe.py)
                } else {
                    const f2 vv = widen_h2(v[p]);
                    s = h2{static_cast<_Float16>(__builtin_amdgcn_sqrtf(vv.x)),
                           static_cast<_Float16>(__builtin_amdgcn_sqrtf(vv.y))};
                }
                const f2 den = widen_h2(u_of(s + tau2));
                const f2 q = {div_rn_h<0>(num[p], den.x), div_rn_h<1>(num[p], den.y)};
                c[p] = u_of(h2_of(c[p]) + h2_of(pk_h2(q)));
            }
        } else {
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                const f2 vv = widen_h2(v[p]), cc = widen_h2(c[p]), nn = widen_h2(num[p]);
                float co[2];
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const float den = f16_round(__fadd_rn(f16_round(__builtin_sqrtf(vv[h])), tau));
                    co[h] = f16_round(__fadd_rn(cc[h], f16_round(__fdiv_rn(nn[h], den))));
                }
                c[p] = u_of(h2{static_cast<_Float16>(co[0]), static_cast<_Float16>(co[1])});   // exact
            }
        }
    };
    auto arrive = [&](const V16& x, float r, bool ends) {
#pragma unroll
        for (int p = 0; p < 4; ++p) b[p] = u_of(h2_of(b[p]) + h2_of(smul_h2(r, x.w[p])));
        if (ends) {     // uniform: one do() call ends here
            if (__builtin_expect(aliased, 0)) {   // the first step after the passthrough: current IS base
#pragma unroll
                for (int p = 0; p < 4; ++p) c[p] = b[p];
                aliased = false;
            }
            adapt();
        }
    };
    auto client = [&](int i) { return reinterpret_cast<const char*>(cp[i]) + coff; };
    int i = 0;
    for (; i + CU <= n_clients; i += CU) {
        V16 x[CU];
        float rr[CU];
        bool ends[CU];
#pragma unroll
        for (int u = 0; u < CU; ++u) x[u] = ld_nt(client(i + u));
#pragma unroll
        for (int u = 0; u < CU; ++u) {
            rr[u] = r32[i + u];
            ends[u] = step_ends(step_end, i + u);
        }
#pragma unroll
        for (int u = 0; u < CU; ++u) arrive(x[u], rr[u], ends[u]);
    }
    for (; i < n_clients; ++i) arrive(ld_nt(client(i)), r32[i], step_ends(step_end, i));
    if (aliased) {             // no step closed: current is still the base
#pragma unroll
        for (int p = 0; p < 4; ++p) c[p] = b[p];
    }
    auto st4 = [](void* p, const uint32_t (&x)[4]) {
        V16 t;
#pragma unroll
        for (int q = 0; q < 4; ++q) t.w[q] = x[q];
        st_v(p, t);
    };
    st4(reinterpret_cast<uint16_t*>(sg.out) + e0, b);
    st4(mp, m);
    st4(vp, v);
    st4(reinterpret_cast<uint16_t*>(sg.cur_out) + e0, c);
}

template <int DT, int VARIANT, int CU>
__global__ __launch_bounds__(kBlock) void fedopt_chain_kernel(const flame_segment* __restrict__ segs, int n_segs,
                                                              const uint64_t* __restrict__ clients, int n_clients,
                                                              const float* __restrict__ r32,
                                                              const uint8_t* __restrict__ step_end, unsigned flags,
                                                              float b1, float omb1, float b2, float omb2, float eta,
                                                              float tau) {
    static_assert(kVPT == 1, "fedopt_chain_kernel: a lane handles one 16-byte vector of its chunk");
    const int64_t chunk = blockIdx.x;
    const int s = find_segment(segs, n_segs, chunk);
    const flame_segment sg = segs[s];
    const int64_t c0 = (chunk - sg.chunk_begin) * chunk_elems<DT>();
    const int64_t e0 = c0 + static_cast<int64_t>(threadIdx.x) * Tr<DT>::EPT;
    if (e0 >= sg.numel) return;
    const uint64_t* cp = clients + static_cast<int64_t>(s) * n_clients;
    const int64_t coff = client_offset<DT>(sg, chunk);
    if (c0 + chunk_elems<DT>() <= sg.numel && !(sg.flags & FLAME_SEG_UNALIGNED)) {   // workgroup-uniform
        if constexpr (DT == FLAME_F16 && kF16Native)
            fedopt_chain_body_f16<VARIANT, CU>(sg, e0, cp, coff, n_clients, r32, step_end, flags, b1, omb1, b2, omb2,
                                               eta, tau);
        else
            fedopt_chain_body<DT, VARIANT, CU, true>(sg, e0, cp, coff, n_clients, r32, step_end, flags, b1, omb1, b2,
                                                     omb2, eta, tau);
    } else
        fedopt_chain_body<DT, VARIANT, 1, false>(sg, e0, cp, coff, n_clients, r32, step_end, flags, b1, omb1, b2,
                                                 omb2, eta, tau);
}

// ---------------------------------------------------------------- FedBuff scale-add (+delta)
template <int DT> struct SA;
template <> struct SA<FLAME_F32> {
    using T = float; static constexpr int EPT = 4;
    __device__ static void op(T& b, T a, float g, double, T* d) {
        const float nb = __fadd_rn(b, __fdiv_rn(a, g));
        if (d) *d = __fsub_rn(nb, b);
        b = nb;
    }
};
template <> struct SA<FLAME_F64> {
    using T = double; static constexpr int EPT = 2;
    __device__ static void op(T& b, T a, float, double g, T* d) {
        const double nb = __dadd_rn(b, __ddiv_rn(a, g));
        if (d) *d = __dsub_rn(nb, b);
        b = nb;
    }
};
template <> struct SA<FLAME_BF16> {
    using T = uint16_t; static constexpr int EPT = 8;
    __device__ static void op(T& b, T a, float g, double, T* d) {
        const float bo = bf16_to_f32(b);
        const float q = bf16_round(__fdiv_rn(bf16_to_f32(a), g));
        const float nb = bf16_round(__fadd_rn(bo, q));
        if (d) *d = f32_to_bf16_exact(bf16_round(__fsub_rn(nb, bo)));
        b = f32_to_bf16_exact(nb);
    }
};
template <> struct SA<FLAME_F16> {
    using T = uint16_t; static constexpr int EPT = 8;
    __device__ static void op(T& b, T a, float g, double, T* d) {
        const float bo = f16_to_f32(b);
        const float q = f16_round(__fdiv_rn(f16_to_f32(a), g));
        const float nb = f16_round(__fadd_rn(bo, q));
        if (d) *d = f32_to_f16_bits(__fsub_rn(nb, bo));
        b = f32_to_f16_bits(nb);
    }
};

template <int DT>
__global__ __launch_bounds__(kEwBlock) void scale_add_kernel(const flame_segment* __restrict__ segs, int n_segs,
                                                           float gf, double gd) {
    using S = SA<DT>;
    using T = typename S::T;
    constexpr int EPT = S::EPT;
    const int64_t chunk = blockIdx.x;
    const int s = find_segment(segs, n_segs, chunk);
    const flame_segment sg = segs[s];
    const int64_t e0 = (chunk - sg.chunk_begin) * (kEwBlock * EPT) + static_cast<int64_t>(threadIdx.x) * EPT;
    if (e0 >= sg.numel) return;
    T* bp = reinterpret_cast<T*>(sg.out) + e0;
    const T* ap = reinterpret_cast<const T*>(sg.in) + e0;
    T* dp = sg.cur_out ? reinterpret_cast<T*>(sg.cur_out) + e0 : nullptr;
    const bool vec = (e0 + EPT <= sg.numel) && !(sg.flags & FLAME_SEG_UNALIGNED);
    if (vec) {
        T b[EPT], a[EPT], d[EPT];
        unpack<T, EPT>(ld_v(bp), b);
        unpack<T, EPT>(ld_v(ap), a);
#pragma unroll
        for (int j = 0; j < EPT; ++j) S::op(b[j], a[j], gf, gd, dp ? &d[j] : nullptr);
        st_v(bp, pack<T, EPT>(b));
        if (dp) st_v(dp, pack<T, EPT>(d));
    } else {
        for (int j = 0; j < EPT; ++j) {
            if (e0 + j >= sg.numel) break;
            T b = ld1(bp + j), d;
            S::op(b, ld1(ap + j), gf, gd, dp ? &d : nullptr);
            st1(bp + j, b);
            if (dp) st1(dp + j, d);
        }
    }
}

// ---------------------------------------------------------------- co-located FedBuff hierarchy
// One pass over a node's whole two-level asynchronous hierarchy:
// for each middle m in the order the top receives their deltas --
//   agg_m  = FedBuff None-start reduce of its C queued arrivals      (fedbuff.py:89-97,136-157)
//   w_m'   = w_m + agg_m / goal_m,  delta_m = w_m' - w_m             (fedbuff.py:122-127,
//                                     asyncfl/middle_aggregator.py:221-226,246, common/util.py:152-159)
//   top    = tmp(delta_m, rate_m) [None start] or top + tmp(...)     (fedbuff.py:96,136-157, top role)
// then top_w += top / top_goal (fedbuff.py:122-127).  Every op rounds in the tensor's
// dtype exactly as the separate launches do, so results are bit-identical to them; the
// middle aggregates and deltas never touch HBM (deltas are stored only if asked for).
// SYNC (FLAME_HIER_SYNC): the synchronous hierarchy instead (syncfl/middle_aggregator.py:163-229,
// syncfl/top_aggregator.py:122-176): each middle's FedAvg starts from its weights,
//   a = w_m + tmp(c_{m,0}, r_{m,0}) + ...;  w_m' = a;  d_m = w_m' - w_m
// and the top's FedAvg adds tmp(d_m, top_rates[m]) to the top weights (top_agg_in).
template <int DT> __device__ __forceinline__ float rnd(float x);
// The element-wise hierarchy (segment tails, misaligned views): the same op sequence as the
// vector paths, one element at a time.
template <int DT, bool SYNC, typename MP>
__device__ __forceinline__ void hier_tail(const flame_hier_segment& sg, int64_t e0, int64_t coff,
                                          const uint64_t* __restrict__ wrow, const uint64_t* __restrict__ drow,
                                          const uint64_t* __restrict__ crow, MP mid_ptr, int n_mids, int n_clients,
                                          const float* __restrict__ mid_rates, const float* __restrict__ mid_goal,
                                          const float* __restrict__ top_rates, float top_goal, unsigned flags) {
    using X = Tr<DT>;
    using S = SA<DT>;
    using T = typename X::T;
    using A = typename X::A;
    constexpr int EPT = X::EPT;
    constexpr int64_t VS = static_cast<int64_t>(kBlock) * EPT;
    (void)wrow;
    A top[kVPT][EPT];
    bool have_top = (flags & FLAME_HIER_TOP_ACCUM) != 0;
    const T* tin = reinterpret_cast<const T*>(sg.top_agg_in) + e0;
#pragma unroll
    for (int v = 0; v < kVPT; ++v)
#pragma unroll
        for (int j = 0; j < EPT; ++j) {
            const int64_t o = v * VS + j;
            if (have_top && e0 + o < sg.numel) top[v][j] = X::ld(ld1(tin + o));
        }
#pragma unroll 1
    for (int m = 0; m < n_mids; ++m) {
        A acc[kVPT][EPT];
        T* wp = mid_ptr(m);
        if constexpr (SYNC) {
#pragma unroll
            for (int v = 0; v < kVPT; ++v)
#pragma unroll
                for (int j = 0; j < EPT; ++j)
                    acc[v][j] = (e0 + v * VS + j < sg.numel) ? X::ld(ld1(wp + v * VS + j)) : A(0);
        }
        reduce_clients<DT, 1, false>(acc, !SYNC, crow + static_cast<int64_t>(m) * n_clients, n_clients,
                                     mid_rates + static_cast<int64_t>(m) * n_clients, nullptr, e0, sg.numel, coff);
        T* dp = (drow && drow[m]) ? reinterpret_cast<T*>(drow[m]) + e0 : nullptr;
        const float g = mid_goal[m], rt = top_rates[m];
#pragma unroll
        for (int v = 0; v < kVPT; ++v)
#pragma unroll
            for (int j = 0; j < EPT; ++j) {
                const int64_t o = v * VS + j;
                if (e0 + o >= sg.numel) continue;
                T w = ld1(wp + o), d;
                if constexpr (SYNC) {
                    const T wn = X::st(acc[v][j]);
                    d = X::st(rnd<DT>(__fsub_rn(X::ld(wn), X::ld(w))));
                    w = wn;
                } else {
                    S::op(w, X::st(acc[v][j]), g, static_cast<double>(g), &d);
                }
                if (!(flags & FLAME_HIER_MID_READONLY)) st1(wp + o, w);
                if (dp) st1(dp + o, d);
                const A t = X::tmp(d, rt, 0.0);
                top[v][j] = have_top ? X::add(top[v][j], t) : t;
            }
        have_top = true;
    }
#pragma unroll
    for (int v = 0; v < kVPT; ++v)
#pragma unroll
        for (int j = 0; j < EPT; ++j) {
            const int64_t o = v * VS + j;
            if (e0 + o >= sg.numel) continue;
            const T t = X::st(top[v][j]);
            if (sg.top_agg_out) st1(reinterpret_cast<T*>(sg.top_agg_out) + e0 + o, t);
            if (flags & FLAME_HIER_TOP_APPLY) {
                T* gp = reinterpret_cast<T*>(sg.top_w) + e0 + o;
                T gw = ld1(gp);
                S::op(gw, t, top_goal, static_cast<double>(top_goal), nullptr);
                st1(gp, gw);
            }
        }
}

// (HL instantiations: the middle loop stays rolled -- its group lives in LDS, not registers)
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Wpass-failed"
template <int DT, int CU, bool SYNC, int HB, bool HL>
__device__ __forceinline__ void hier_fedbuff_body(const flame_hier_segment* __restrict__ segs, int n_segs,
                                                  int n_mids, int n_clients, const uint64_t* __restrict__ mid_w,
                                                  const uint64_t* __restrict__ mid_delta,
                                                  const uint64_t* __restrict__ clients,
                                                  const float* __restrict__ mid_rates,
                                                  const float* __restrict__ mid_goal,
                                                  const float* __restrict__ top_rates, float top_goal,
                                                  unsigned flags) {
    using X = Tr<DT>;
    using S = SA<DT>;
    using T = typename X::T;
    using A = typename X::A;
    constexpr int EPT = X::EPT;
    constexpr int64_t VS = static_cast<int64_t>(kBlock) * EPT;
    const int64_t chunk = blockIdx.x;
    const int s = find_segment(segs, n_segs, chunk);
    const flame_hier_segment sg = segs[s];
    const int64_t e0 = (chunk - sg.chunk_begin) * chunk_elems<DT>() + static_cast<int64_t>(threadIdx.x) * EPT;
    if (e0 >= sg.numel) return;
    const int64_t coff = client_offset<DT>(sg, chunk);
    const uint64_t* wrow = mid_w + static_cast<int64_t>(s) * n_mids;
    const uint64_t* drow = mid_delta ? mid_delta + static_cast<int64_t>(s) * n_mids : nullptr;
    const uint64_t* crow = clients + static_cast<int64_t>(s) * n_mids * n_clients;
    const bool vec = (e0 + (kVPT - 1) * VS + EPT <= sg.numel) && !(sg.flags & FLAME_SEG_UNALIGNED);
    // byte offset of this lane's elements inside every middle's weights: contiguous or tiled
    const int64_t woff = sg.mid_tile_stride
        ? (chunk - sg.chunk_begin) * sg.mid_tile_stride + static_cast<int64_t>(threadIdx.x) * EPT * sizeof(T)
        : e0 * static_cast<int64_t>(sizeof(T));
    auto mid_ptr = [&](int m) { return reinterpret_cast<T*>(reinterpret_cast<char*>(wrow[m]) + woff); };
    A top[kVPT][EPT];
    bool have_top = (flags & FLAME_HIER_TOP_ACCUM) != 0;
    const T* tin = reinterpret_cast<const T*>(sg.top_agg_in) + e0;
    if (vec) {
        if (have_top) {
#pragma unroll
            for (int v = 0; v < kVPT; ++v) {
                T b[EPT];
                unpack<T, EPT>(ld_v(tin + v * VS), b);
#pragma unroll
                for (int j = 0; j < EPT; ++j) top[v][j] = X::ld(b[j]);
            }
        }
        // middles in groups of HB: a group's middle-weight stores are issued together after its
        // reductions (1 = store each middle's weights right after its reduction).  HL: the group's
        // weights wait in LDS (lane-private slots, no barrier) rather than in registers -- long
        // store bursts at 2 workgroups per CU
        __shared__ V16 held[HL ? HB * kVPT * kBlock : 1];
#pragma unroll 1
        for (int m0 = 0; m0 < n_mids; m0 += HB) {
            V16 pend[HL ? 1 : HB][kVPT];
            const int nb = n_mids - m0 < HB ? n_mids - m0 : HB;   // middles in this group
#pragma unroll
            for (int u = 0; u < HB; ++u) {
            const int m = m0 + u;
            if (HB > 1 && m >= n_mids) break;
            T* wp = mid_ptr(m);
            A acc[kVPT][EPT];
            T wo[SYNC ? kVPT : 1][EPT];
            if constexpr (SYNC) {     // FedAvg starts from the middle's weights (deepcopy(self.weights))
#pragma unroll
                for (int v = 0; v < kVPT; ++v) {
                    unpack<T, EPT>(ld_v(wp + v * VS), wo[v]);
#pragma unroll
                    for (int j = 0; j < EPT; ++j) acc[v][j] = X::ld(wo[v][j]);
                }
            }
            reduce_clients<DT, CU, true>(acc, !SYNC, crow + static_cast<int64_t>(m) * n_clients, n_clients,
                                         mid_rates + static_cast<int64_t>(m) * n_clients, nullptr, e0, sg.numel,
                                         coff);
            T* dp = (drow && drow[m]) ? reinterpret_cast<T*>(drow[m]) + e0 : nullptr;
            const float g = mid_goal[m], rt = top_rates[m];
#pragma unroll
            for (int v = 0; v < kVPT; ++v) {
                T w[EPT], d[EPT];
                if constexpr (SYNC) {
#pragma unroll
                    for (int j = 0; j < EPT; ++j) {
                        w[j] = X::st(acc[v][j]);
                        d[j] = X::st(rnd<DT>(__fsub_rn(X::ld(w[j]), X::ld(wo[v][j]))));
                        top[v][j] = X::add(top[v][j], X::tmp(d[j], rt, 0.0));
                    }
                } else {
                    unpack<T, EPT>(ld_v(wp + v * VS), w);
#pragma unroll
                    for (int j = 0; j < EPT; ++j) {
                        S::op(w[j], X::st(acc[v][j]), g, static_cast<double>(g), &d[j]);
                        const A t = X::tmp(d[j], rt, 0.0);
                        top[v][j] = have_top ? X::add(top[v][j], t) : t;
                    }
                }
                if constexpr (HL) held[(u * kVPT + v) * kBlock + threadIdx.x] = pack<T, EPT>(w);
                else pend[u][v] = pack<T, EPT>(w);
                if (dp) st_v(dp + v * VS, pack<T, EPT>(d));
            }
            have_top = true;
            }
            if (!(flags & FLAME_HIER_MID_READONLY)) {
#pragma unroll
                for (int u = 0; u < HB; ++u) {
                    if (u >= nb) break;
                    T* wp = mid_ptr(m0 + u);       // re-read from the (scalar) pointer table
#pragma unroll
                    for (int v = 0; v < kVPT; ++v) {
                        V16 pv;
                        if constexpr (HL) pv = held[(u * kVPT + v) * kBlock + threadIdx.x];
                        else pv = pend[u][v];
                        st_v(wp + v * VS, pv);
                    }
                }
            }
        }
#pragma unroll
        for (int v = 0; v < kVPT; ++v) {
            T o[EPT];
#pragma unroll
            for (int j = 0; j < EPT; ++j) o[j] = X::st(top[v][j]);
            if (sg.top_agg_out) st_v(reinterpret_cast<T*>(sg.top_agg_out) + e0 + v * VS, pack<T, EPT>(o));
            if (flags & FLAME_HIER_TOP_APPLY) {
                T* gp = reinterpret_cast<T*>(sg.top_w) + e0 + v * VS;
                T gw[EPT];
                unpack<T, EPT>(ld_v(gp), gw);
#pragma unroll
                for (int j = 0; j < EPT; ++j) S::op(gw[j], o[j], top_goal, static_cast<double>(top_goal), nullptr);
                st_v(gp, pack<T, EPT>(gw));
            }
        }
        return;
    }
    hier_tail<DT, SYNC>(sg, e0, coff, wrow, drow, crow, mid_ptr, n_mids, n_clients, mid_rates, mid_goal, top_rates,
                        top_goal, flags);
}

template <int DT, int CU, bool SYNC, int HB, bool HL>
__global__ __launch_bounds__(kBlock) void hier_fedbuff_kernel(const flame_hier_segment* __restrict__ segs, int n_segs,
                                                    int n_mids, int n_clients, const uint64_t* __restrict__ mid_w,
                                                    const uint64_t* __restrict__ mid_delta,
                                                    const uint64_t* __restrict__ clients,
                                                    const float* __restrict__ mid_rates,
                                                    const float* __restrict__ mid_goal,
                                                    const float* __restrict__ top_rates, float top_goal,
                                                    unsigned flags) {
    hier_fedbuff_body<DT, CU, SYNC, HB, HL>(segs, n_segs, n_mids, n_clients, mid_w, mid_delta, clients, mid_rates, mid_goal,
                                    top_rates, top_goal, flags);
}

// The same with the metadata block in the kernel arguments (small launches, e.g. a single
// FedBuff aggregator's fused scale_add); word offsets into the block, -1 = no delta table.
template <int DT, int CU, bool SYNC, int HB, bool HL>
__global__ __launch_bounds__(kBlock) void hier_fedbuff_kernel_argmeta(const ArgMeta meta, int n_segs, int n_mids, int n_clients,
                                                            int o_mid_w, int o_mid_delta, int o_clients,
                                                            int o_mid_rates, int o_mid_goal, int o_top_rates,
                                                            float top_goal, unsigned flags) {
    (void)sizeof(meta);     // read in place in the kernarg segment (see agg_reduce_kernel_argmeta)
    const uint64_t* w = (const uint64_t*)__builtin_amdgcn_kernarg_segment_ptr();
    hier_fedbuff_body<DT, CU, SYNC, HB, HL>(reinterpret_cast<const flame_hier_segment*>(w), n_segs, n_mids, n_clients,
                                    w + o_mid_w, o_mid_delta >= 0 ? w + o_mid_delta : nullptr, w + o_clients,
                                    reinterpret_cast<const float*>(w + o_mid_rates),
                                    reinterpret_cast<const float*>(w + o_mid_goal),
                                    reinterpret_cast<const float*>(w + o_top_rates), top_goal, flags);
}
#pragma clang diagnostic pop

// ---------------------------------------------------------------- FedDyn server round
// One pass over a FedDyn aggregation round (optimizer/feddyn.py:90-113,125-139), driven
// by a host-built step program.  Per element, in step order (every op rounded in dtype):
//   W:    load the arrival w (tiled or contiguous, like flame_agg_reduce's clients)
//   HIN:  load a history h (contiguous)
//   AVG:  avg = avg + tmp(w, r_avg)                           (FedAvg, rate 1/len(cache))
//   HOUT: h' = HIN ? h + w : w, stored to h_out               (add_to_hist)
//   MEAN: mean = mean + tmp(HOUT ? h' : h, r_mean), mean0 = +0 (0.0 + Σ rate*h)
// then out = avg, cld = avg + mean.  Steps [0, n_phase1) run before [n_phase1, n_steps);
// batched loads never cross that boundary, so a phase-2 step may re-read what a phase-1
// step stored (history order != arrival order).
template <int DT, int CU, bool VEC>
__device__ __forceinline__ void feddyn_chunk(const flame_dyn_segment& sg, const uint64_t* __restrict__ row,
                                             const uint32_t* __restrict__ sflags, int n_steps, int n_phase1,
                                             float ra32, float rm32, double ra64, double rm64, int64_t e0,
                                             int64_t coff, int64_t hoff) {
    using X = Tr<DT>;
    using T = typename X::T;
    using A = typename X::A;
    constexpr int EPT = X::EPT;
    constexpr int64_t VS = static_cast<int64_t>(kBlock) * EPT;
    const int64_t ooff = e0 * static_cast<int64_t>(sizeof(T));   // base / average / cld: contiguous
    auto load = [&](uint64_t base, int64_t off, T (&x)[kVPT][EPT]) {
        const T* p = reinterpret_cast<const T*>(reinterpret_cast<const char*>(base) + off);
#pragma unroll
        for (int v = 0; v < kVPT; ++v) {
            if constexpr (VEC) {
                unpack<T, EPT>(ld_nt(p + v * VS), x[v]);
            } else {
#pragma unroll
                for (int j = 0; j < EPT; ++j) x[v][j] = (e0 + v * VS + j < sg.numel) ? ld1(p + v * VS + j) : T(0);
            }
        }
    };
    auto store = [&](void* base, int64_t off, const T (&x)[kVPT][EPT]) {
        T* p = reinterpret_cast<T*>(reinterpret_cast<char*>(base) + off);
#pragma unroll
        for (int v = 0; v < kVPT; ++v) {
            if constexpr (VEC) {
                st_v(p + v * VS, pack<T, EPT>(x[v]));
            } else {
#pragma unroll
                for (int j = 0; j < EPT; ++j)
                    if (e0 + v * VS + j < sg.numel) st1(p + v * VS + j, x[v][j]);
            }
        }
    };
    A avg[kVPT][EPT], mean[kVPT][EPT];
    {
        T b[kVPT][EPT];
        load(reinterpret_cast<uint64_t>(sg.in), ooff, b);
#pragma unroll
        for (int v = 0; v < kVPT; ++v)
#pragma unroll
            for (int j = 0; j < EPT; ++j) { avg[v][j] = X::ld(b[v][j]); mean[v][j] = A(0); }
    }
#pragma unroll 1
    for (int phase = 0; phase < 2; ++phase) {
        const int end = phase ? n_steps : n_phase1;
#pragma unroll 1
        for (int k = phase ? n_phase1 : 0; k < end; k += CU) {
            const int nb = (end - k < CU) ? end - k : CU;
            T w[CU][kVPT][EPT], h[CU][kVPT][EPT];
#pragma unroll
            for (int u = 0; u < CU; ++u) {
                if (u >= nb) break;
                const uint32_t f = sflags[k + u];
                const uint64_t* p = row + static_cast<int64_t>(k + u) * 3;
                if (f & FLAME_DYN_W) load(p[0], coff, w[u]);
                if (f & FLAME_DYN_HIN) load(p[1], hoff, h[u]);
            }
#pragma unroll
            for (int u = 0; u < CU; ++u) {
                if (u >= nb) break;
                const uint32_t f = sflags[k + u];
                if (f & FLAME_DYN_AVG) {
#pragma unroll
                    for (int v = 0; v < kVPT; ++v)
#pragma unroll
                        for (int j = 0; j < EPT; ++j) avg[v][j] = X::add(avg[v][j], X::tmp(w[u][v][j], ra32, ra64));
                }
                if (f & FLAME_DYN_HOUT) {
                    if (f & FLAME_DYN_HIN) {
#pragma unroll
                        for (int v = 0; v < kVPT; ++v)
#pragma unroll
                            for (int j = 0; j < EPT; ++j) h[u][v][j] = X::st(X::add(X::ld(h[u][v][j]), X::ld(w[u][v][j])));
                    } else {
#pragma unroll
                        for (int v = 0; v < kVPT; ++v)
#pragma unroll
                            for (int j = 0; j < EPT; ++j) h[u][v][j] = w[u][v][j];
                    }
                    store(reinterpret_cast<void*>(row[static_cast<int64_t>(k + u) * 3 + 2]), hoff, h[u]);
                }
                if (f & FLAME_DYN_MEAN) {
#pragma unroll
                    for (int v = 0; v < kVPT; ++v)
#pragma unroll
                        for (int j = 0; j < EPT; ++j) mean[v][j] = X::add(mean[v][j], X::tmp(h[u][v][j], rm32, rm64));
                }
            }
        }
    }
    T o[kVPT][EPT], c[kVPT][EPT];
#pragma unroll
    for (int v = 0; v < kVPT; ++v)
#pragma unroll
        for (int j = 0; j < EPT; ++j) { o[v][j] = X::st(avg[v][j]); c[v][j] = X::st(X::add(avg[v][j], mean[v][j])); }
    store(sg.out, ooff, o);
    store(sg.cld, ooff, c);
}

template <int DT, int CU>
__global__ __launch_bounds__(kBlock) void feddyn_kernel(const flame_dyn_segment* __restrict__ segs, int n_segs,
                                                        const uint64_t* __restrict__ steps,
                                                        const uint32_t* __restrict__ sflags, int n_steps,
                                                        int n_phase1, float ra32, float rm32, double ra64,
                                                        double rm64) {
    using X = Tr<DT>;
    constexpr int EPT = X::EPT;
    constexpr int64_t VS = static_cast<int64_t>(kBlock) * EPT;
    // XCD-contiguous chunk map: 512 x 12M fp32 -0.7 % (cache order) / -1.4 % (other order)
    // (profiles/r02_feddyn_xcd_sweep.log)
    const int64_t chunk = xcd_slot(blockIdx.x, gridDim.x);
    const int s = find_segment(segs, n_segs, chunk);
    const flame_dyn_segment sg = segs[s];
    const int64_t e0 = (chunk - sg.chunk_begin) * chunk_elems<DT>() + static_cast<int64_t>(threadIdx.x) * EPT;
    if (e0 >= sg.numel) return;
    const int64_t coff = client_offset<DT>(sg, chunk);
    // histories: contiguous, or tiled like the arrivals (a FedDyn history store in the slab layout)
    const int64_t hoff = sg.hist_tile_stride
        ? (chunk - sg.chunk_begin) * sg.hist_tile_stride + static_cast<int64_t>(threadIdx.x) * EPT * static_cast<int64_t>(sizeof(typename X::T))
        : e0 * static_cast<int64_t>(sizeof(typename X::T));
    const uint64_t* row = steps + static_cast<int64_t>(s) * n_steps * 3;
    const bool vec = (e0 + (kVPT - 1) * VS + EPT <= sg.numel) && !(sg.flags & FLAME_SEG_UNALIGNED);
    if (vec)
        feddyn_chunk<DT, CU, true>(sg, row, sflags, n_steps, n_phase1, ra32, rm32, ra64, rm64, e0, coff, hoff);
    else
        feddyn_chunk<DT, 1, false>(sg, row, sflags, n_steps, n_phase1, ra32, rm32, ra64, rm64, e0, coff, hoff);
}

// ---------------------------------------------------------------- synthetic generator
__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

template <int DT>
__global__ __launch_bounds__(kEwBlock) void synth_kernel(void* out, int64_t numel, uint64_t ck, int64_t start, float scale) {
    const int64_t stride = static_cast<int64_t>(gridDim.x) * kEwBlock;
    for (int64_t j = static_cast<int64_t>(blockIdx.x) * kEwBlock + threadIdx.x; j < numel; j += stride) {
        const uint64_t h = mix64(ck + static_cast<uint64_t>(start + j) * 0x9E3779B97F4A7C15ull);
        const int32_t s = static_cast<int32_t>((h & 0xFFFFu) + ((h >> 16) & 0xFFFFu) + ((h >> 32) & 0xFFFFu) + (h >> 48)) - 131070;
        const float x = __fmul_rn(static_cast<float>(s), scale);
        if constexpr (DT == FLAME_F32) st1(reinterpret_cast<float*>(out) + j, x);
        else if constexpr (DT == FLAME_BF16) st1(reinterpret_cast<uint16_t*>(out) + j, f32_to_bf16_exact(bf16_round(x)));
        else st1(reinterpret_cast<uint16_t*>(out) + j, f32_to_f16_bits(x));
    }
}

// ---------------------------------------------------------------- slab insert (tiling copy)
// The role's `self.cache[end] = tres` (syncfl/top_aggregator.py:154-156) lands one update
// in a slab slot: each key's contiguous bytes are cut into 4 KiB tiles (one reduction
// chunk of any dtype) written `dst_tile_stride` apart (the slab's capacity x 4 KiB).  One
// workgroup copies kSlabTPW tiles, every lane 16 B of each (all its loads issued before its
// stores); the entry table rides in the kernel arguments, so an insert is ONE launch and no
// H2D of metadata.
// 2 tiles per workgroup (1-8 within noise) and plain stores (measured best of the store policies,
// profiles/r03b_slab_sweep.log)
constexpr int kSlabTPW = 2;
struct SlabEntry { const uint8_t* src; uint8_t* dst; int64_t nbytes; int64_t stride; int64_t tile_begin; };
constexpr int kSlabMaxEntries = static_cast<int>(sizeof(ArgMeta) / sizeof(SlabEntry));
static_assert(FLAME_TILE_BYTES == kBlock * 16, "a slab tile is one 16-byte vector per lane");

__global__ __launch_bounds__(kBlock) void slab_write_kernel(const ArgMeta meta, int n_entries, int64_t n_tiles) {
    (void)sizeof(meta);
    const SlabEntry* ents = (const SlabEntry*)__builtin_amdgcn_kernarg_segment_ptr();
    const int lane = threadIdx.x;
    V16 v[kSlabTPW];
    uint8_t* dp[kSlabTPW];
    int kind[kSlabTPW];   // 0 none, 1 vector, 2 bytes
#pragma unroll
    for (int j = 0; j < kSlabTPW; ++j) {
        const int64_t tile = static_cast<int64_t>(blockIdx.x) * kSlabTPW + j;
        kind[j] = 0;
        dp[j] = nullptr;
        if (tile >= n_tiles) continue;
        int lo = 0, hi = n_entries - 1;           // wave-uniform: last entry with tile_begin <= tile
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (ents[mid].tile_begin <= tile) lo = mid; else hi = mid - 1;
        }
        const SlabEntry& e = ents[lo];
        const int64_t t = tile - e.tile_begin;
        const int64_t off = t * FLAME_TILE_BYTES + lane * 16;
        if (off >= e.nbytes) continue;
        dp[j] = e.dst + t * e.stride + lane * 16;
        const uint8_t* sp = e.src + off;
        const int sh = static_cast<int>(reinterpret_cast<uintptr_t>(sp) & 15);   // uniform per entry
        if (off + 16 <= e.nbytes && sh == 0) {
            v[j] = ld_nt(sp);
            kind[j] = 1;
        } else if (off + 16 <= e.nbytes) {
            // misaligned source (e.g. tensor bytes inside a channel payload): two aligned loads
            // and a byte funnel shift.  The second 16-byte block starts before the entry's last
            // byte, so it never leaves that byte's (4 KiB-aligned) page.
            const uint8_t* ab = sp - sh;
            const V16 lo = ld_nt(ab), hi = ld_nt(ab + 16);
            const uint32_t w[8] = {lo.w[0], lo.w[1], lo.w[2], lo.w[3], hi.w[0], hi.w[1], hi.w[2], hi.w[3]};
            const unsigned r = static_cast<unsigned>(sh & 3);
#define FLAME_SLAB_FUNNEL(Q) \
    for (int i = 0; i < 4; ++i) v[j].w[i] = __builtin_amdgcn_alignbyte(w[i + (Q) + 1], w[i + (Q)], r);
            switch (sh >> 2) {
            case 0: FLAME_SLAB_FUNNEL(0) break;
            case 1: FLAME_SLAB_FUNNEL(1) break;
            case 2: FLAME_SLAB_FUNNEL(2) break;
            default: FLAME_SLAB_FUNNEL(3) break;
            }
#undef FLAME_SLAB_FUNNEL
            kind[j] = 1;
        } else {                                  // ragged tail
            const int nb = static_cast<int>(e.nbytes - off < 16 ? e.nbytes - off : 16);
            for (int b = 0; b < nb; ++b) st1(dp[j] + b, ld1(sp + b));
            kind[j] = 2;
        }
    }
#pragma unroll
    for (int j = 0; j < kSlabTPW; ++j)
        if (kind[j] == 1) st_plain(dp[j], v[j]);
}

// ---------------------------------------------------------------- elementwise programs
// flame_elementwise (include/flame_amd.h): the reference's torch statements for keys the fused
// kernels do not take -- an int buffer (num_batches_tracked), a mixed-dtype or fp64 key -- as a
// short typed op list read from the kernel arguments in place (scalar loads; every wave takes the
// same switch arm).  A register holds a double (every fp32 / bf16 / fp16 value is exact in one)
// or an int64.  Such keys are small, so the registers may live in scratch.
struct EwArgs {
    flame_ew_op ops[FLAME_EW_MAX_OPS];
    void* bufs[FLAME_EW_MAX_BUFS];       // one segment: the buffers
    void* const* table;                  // segments: device [n_segs][n_bufs] buffers (else NULL)
    const int64_t* seg_end;              // segments: device [n_segs] inclusive element prefix sums
    int64_t numel;
    int32_t n_ops, n_segs, n_bufs;
};
union EwVal {
    double f;
    int64_t i;
};

__host__ __device__ __forceinline__ bool ew_float(int dt) { return dt >= FLAME_F32 && dt <= FLAME_F64; }
// an fp32 result into a 32-bit-or-narrower float dtype (torch's opmath result, rounded once)
__device__ __forceinline__ double ew_rnd32(float x, int dt) {
    if (dt == FLAME_BF16) return bf16_round(x);
    if (dt == FLAME_F16) return f16_round(x);
    return x;
}
// an int64 wrapped to the integer dtype's width (two's complement, as torch's int ops wrap)
__device__ __forceinline__ int64_t ew_wrap(int64_t x, int dt) {
    switch (dt) {
    case FLAME_I32: return static_cast<int32_t>(static_cast<uint32_t>(x));
    case FLAME_I16: return static_cast<int16_t>(static_cast<uint16_t>(x));
    case FLAME_I8: return static_cast<int8_t>(static_cast<uint8_t>(x));
    case FLAME_U8: return static_cast<uint8_t>(x);
    case FLAME_BOOL: return x != 0;
    default: return x;
    }
}
__device__ __forceinline__ EwVal ew_load(const void* p, int64_t i, int dt) {
    EwVal v;
    switch (dt) {
    case FLAME_F32: v.f = ld1(static_cast<const float*>(p) + i); break;
    case FLAME_BF16: v.f = bf16_to_f32(ld1(static_cast<const uint16_t*>(p) + i)); break;
    case FLAME_F16: v.f = f16_to_f32(ld1(static_cast<const uint16_t*>(p) + i)); break;
    case FLAME_F64: v.f = ld1(static_cast<const double*>(p) + i); break;
    case FLAME_I64: v.i = ld1(static_cast<const int64_t*>(p) + i); break;
    case FLAME_I32: v.i = ld1(static_cast<const int32_t*>(p) + i); break;
    case FLAME_I16: v.i = ld1(static_cast<const int16_t*>(p) + i); break;
    case FLAME_I8: v.i = ld1(static_cast<const int8_t*>(p) + i); break;
    default: v.i = ld1(static_cast<const uint8_t*>(p) + i); break;        // U8, BOOL
    }
    return v;
}
__device__ __forceinline__ void ew_store(void* p, int64_t i, int dt, EwVal v) {
    switch (dt) {
    case FLAME_F32: st1(static_cast<float*>(p) + i, static_cast<float>(v.f)); break;
    case FLAME_BF16: st1(static_cast<uint16_t*>(p) + i, f32_to_bf16_exact(static_cast<float>(v.f))); break;
    case FLAME_F16: st1(static_cast<uint16_t*>(p) + i, f32_to_f16_bits(static_cast<float>(v.f))); break;
    case FLAME_F64: st1(static_cast<double*>(p) + i, v.f); break;
    case FLAME_I64: st1(static_cast<int64_t*>(p) + i, v.i); break;
    case FLAME_I32: st1(static_cast<int32_t*>(p) + i, static_cast<int32_t>(v.i)); break;
    case FLAME_I16: st1(static_cast<int16_t*>(p) + i, static_cast<int16_t>(v.i)); break;
    case FLAME_I8: st1(static_cast<int8_t*>(p) + i, static_cast<int8_t>(v.i)); break;
    default: st1(static_cast<uint8_t*>(p) + i, static_cast<uint8_t>(v.i)); break;
    }
}
// CAST from dtype s to dtype t (c10's conversions: an int or an fp64 value reaches bf16 / fp16
// through fp32; a float reaches an int toward zero)
__device__ __forceinline__ EwVal ew_cast(EwVal x, int s, int t) {
    EwVal r;
    if (ew_float(t)) {
        if (t == FLAME_F64) r.f = ew_float(s) ? x.f : __ll2double_rn(x.i);
        else {
            const float f = ew_float(s) ? (s == FLAME_F64 ? __double2float_rn(x.f) : static_cast<float>(x.f))
                                        : __ll2float_rn(x.i);
            r.f = ew_rnd32(f, t);
        }
    } else if (t == FLAME_BOOL) {
        r.i = ew_float(s) ? (x.f != 0.0) : (x.i != 0);
    } else {
        r.i = ew_wrap(ew_float(s) ? __double2ll_rz(x.f) : x.i, t);
    }
    return r;
}
// a binary op in dtype dt on two values of dt (fp32 opmath for bf16 / fp16, as torch-CPU)
template <int OP>
__device__ __forceinline__ EwVal ew_bin(EwVal a, EwVal b, int dt) {
    EwVal r;
    if (dt == FLAME_F64) {
        r.f = OP == FLAME_EW_ADD ? __dadd_rn(a.f, b.f) : OP == FLAME_EW_SUB ? __dsub_rn(a.f, b.f)
            : OP == FLAME_EW_MUL ? __dmul_rn(a.f, b.f) : flame_fm::ddiv_rn(a.f, b.f);
    } else if (ew_float(dt)) {
        const float x = static_cast<float>(a.f), y = static_cast<float>(b.f);
        r.f = ew_rnd32(OP == FLAME_EW_ADD ? __fadd_rn(x, y) : OP == FLAME_EW_SUB ? __fsub_rn(x, y)
                       : OP == FLAME_EW_MUL ? __fmul_rn(x, y) : __fdiv_rn(x, y), dt);
    } else {
        const uint64_t x = static_cast<uint64_t>(a.i), y = static_cast<uint64_t>(b.i);
        r.i = ew_wrap(static_cast<int64_t>(OP == FLAME_EW_ADD ? x + y : OP == FLAME_EW_SUB ? x - y : x * y), dt);
    }
    return r;
}

// (The registers live in a private array, which the dynamic indexing puts in scratch; held in LDS
// instead, [register][lane], a 25M-element fp64 FedAdam step ran slower: 1.520 vs 1.407 ms,
// profiles/r06zh_ew_fp64_lds.log.)
// One op of a program on one element (registers r, the element's buffers and index).
__device__ __forceinline__ void ew_step(const flame_ew_op& o, EwVal* r, void* const* bufs, int64_t i) {
    const int dt = o.dtype;
    switch (o.op) {
    case FLAME_EW_LOAD: r[o.dst] = ew_load(bufs[o.a], i, dt); break;
    case FLAME_EW_STORE: ew_store(bufs[o.a], i, dt, r[o.b]); break;
    case FLAME_EW_ZERO: if (ew_float(dt)) r[o.dst].f = 0.0; else r[o.dst].i = 0; break;
    case FLAME_EW_CAST: r[o.dst] = ew_cast(r[o.a], o.b, dt); break;
    case FLAME_EW_ADD: r[o.dst] = ew_bin<FLAME_EW_ADD>(r[o.a], r[o.b], dt); break;
    case FLAME_EW_SUB: r[o.dst] = ew_bin<FLAME_EW_SUB>(r[o.a], r[o.b], dt); break;
    case FLAME_EW_MUL: r[o.dst] = ew_bin<FLAME_EW_MUL>(r[o.a], r[o.b], dt); break;
    case FLAME_EW_DIV: r[o.dst] = ew_bin<FLAME_EW_DIV>(r[o.a], r[o.b], dt); break;
    case FLAME_EW_ADD_S:
    case FLAME_EW_MUL_S: {
        EwVal s;
        if (dt == FLAME_F64) s.f = o.scalar;
        else if (ew_float(dt)) {
            // torch-CPU: a Python scalar multiplies a float tensor in fp32 (opmath) but is
            // rounded to a bf16 / fp16 tensor's dtype before it is added
            const float sf = __double2float_rn(o.scalar);
            s.f = o.op == FLAME_EW_ADD_S ? ew_rnd32(sf, dt) : sf;
        } else {
            s.i = __double2ll_rz(o.scalar);
        }
        r[o.dst] = o.op == FLAME_EW_ADD_S ? ew_bin<FLAME_EW_ADD>(r[o.a], s, dt) : ew_bin<FLAME_EW_MUL>(r[o.a], s, dt);
        break;
    }
    case FLAME_EW_SQUARE: r[o.dst] = ew_bin<FLAME_EW_MUL>(r[o.a], r[o.a], dt); break;
    case FLAME_EW_SIGN: {
        EwVal v = r[o.a];
        if (ew_float(dt)) v.f = static_cast<double>((0.0 < v.f) - (v.f < 0.0));   // NaN, -0 -> +0
        else v.i = (v.i > 0) - (v.i < 0);
        r[o.dst] = v;
        break;
    }
    case FLAME_EW_SQRT: {
        EwVal v = r[o.a];
        if (dt == FLAME_F64) v.f = flame_fm::dsqrt_rn(v.f);
        else v.f = ew_rnd32(__builtin_sqrtf(static_cast<float>(v.f)), dt);   // correctly rounded
        r[o.dst] = v;
        break;
    }
    default: break;
    }
}

// One element per lane per pass over the program: two or four (the op fetch and dispatch paid
// once for several) ran slower, 1.616 / 1.757 vs 1.411 ms per 25M-element fp64 FedAdam step
// (profiles/r06zi_ew_fp64_ilp.log) -- more registers in scratch; so did registers in LDS (1.520).
__global__ __launch_bounds__(kEwBlock) void ew_kernel(EwArgs args) {
    (void)sizeof(args);      // read in place from the kernarg segment (see agg_reduce_kernel_argmeta)
    const EwArgs* P = (const EwArgs*)__builtin_amdgcn_kernarg_segment_ptr();
    const int64_t numel = P->numel;
    const int n_ops = P->n_ops;
    const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
    void* const* table = P->table;
    for (int64_t g = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; g < numel; g += stride) {
        // the element's segment (several keys of one program in one launch) and index in it
        int64_t i = g;
        void* const* bufs = P->bufs;
        if (table) {
            int lo = 0, hi = P->n_segs - 1;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (P->seg_end[mid] > g) hi = mid; else lo = mid + 1;
            }
            i = g - (lo ? P->seg_end[lo - 1] : 0);
            bufs = table + static_cast<int64_t>(lo) * P->n_bufs;
        }
        EwVal r[FLAME_EW_MAX_REGS];
        for (int k = 0; k < n_ops; ++k) ew_step(P->ops[k], r, bufs, i);
    }
}

// ---------------------------------------------------------------- launch-branch counters
// Every host-side launch branch of the C ABI has an index; a successful launch counts it, so
// tests can assert which instantiation a call took and that every branch is reached by an
// oracle test (tests/test_gpu_zz_launch_branches.py).  dt = FLAME_F32 .. FLAME_I32.
enum : int {
    BR_AGG = 0,           // + dt (6): flame_agg_reduce, full residency
    BR_AGG_LO = 6,        // + dt (f32, bf16, f16): flame_agg_reduce, 2 workgroups per CU
    BR_AGG_ARG = 9,       // + dt (6): flame_agg_reduce_argmeta
    BR_OPT = 15,          // + dt * 3 + variant (f32, bf16, f16): flame_fedopt_reduce_adapt, one chunk per workgroup
    BR_OPT_MULTI = 24,    // + variant: fp32, kOptWGC chunks per workgroup
    BR_OPT_ARG = 27,      // + dt * 3 + variant: flame_fedopt_reduce_adapt_argmeta
    BR_SA = 36,           // + dt (f32, bf16, f16, f64): flame_fedbuff_scale_add
    BR_HIER_REG = 40,     // + dt * 2 + sync: flame_hier_fedbuff, register store groups
    BR_HIER_LDS = 46,     // + dt * 2 + sync: LDS store groups (>= kHLdsMinMids middles)
    BR_HIER_LO = 52,      // + dt: one middle over a long launch, low residency (FedBuff only)
    BR_HIER_ARG = 55,     // + dt * 2 + sync: flame_hier_fedbuff_argmeta
    BR_DYN = 61,          // + dt (f32, bf16, f16, f64): flame_feddyn_round
    BR_AGG_ARG_LO = 65,   // + dt (f32, bf16, f16): flame_agg_reduce_argmeta, 2 workgroups per CU, output bursts
    BR_HIER_ARG_LO = 68,  // + dt: flame_hier_fedbuff_argmeta, one middle over a long launch
    BR_OPT_ARG_MULTI = 71,  // + variant: flame_fedopt_reduce_adapt_argmeta, fp32, kOptWGC chunks per workgroup
    BR_HIER_ARG_LDS = 74,   // + dt * 2 + sync: flame_hier_fedbuff_argmeta, LDS store groups
    BR_CHAIN = 80,          // + dt * 3 + variant (f32, bf16, f16): flame_fedopt_chain
    BR_AGG_LOB = 89,        // + dt (f32, bf16, f16): flame_agg_reduce, low residency, LDS-held output bursts
    BR_EW = 92,             // flame_elementwise
    BR_EW_SEG = 93,         // flame_elementwise_segments
    BR_COUNT = 94
};
std::atomic<long long> g_launches[BR_COUNT];

const char* branch_name(int i) {
    static const char* const dts[6] = {"f32", "bf16", "f16", "f64", "i64", "i32"};
    static const char* const var[3] = {"fedadam", "fedyogi", "fedadagrad"};
    static char names[BR_COUNT][64];
    static const bool once = [] {
        for (int b = 0; b < BR_COUNT; ++b) {
            char* n = names[b];
            const size_t z = sizeof(names[b]);
            if (b < BR_AGG_LO) snprintf(n, z, "flame_agg_reduce/%s", dts[b - BR_AGG]);
            else if (b < BR_AGG_ARG) snprintf(n, z, "flame_agg_reduce/lo/%s", dts[b - BR_AGG_LO]);
            else if (b < BR_OPT) snprintf(n, z, "flame_agg_reduce_argmeta/%s", dts[b - BR_AGG_ARG]);
            else if (b < BR_OPT_MULTI) snprintf(n, z, "flame_fedopt_reduce_adapt/%s/%s", dts[(b - BR_OPT) / 3], var[(b - BR_OPT) % 3]);
            else if (b < BR_OPT_ARG) snprintf(n, z, "flame_fedopt_reduce_adapt/multi/f32/%s", var[b - BR_OPT_MULTI]);
            else if (b < BR_SA) snprintf(n, z, "flame_fedopt_reduce_adapt_argmeta/%s/%s", dts[(b - BR_OPT_ARG) / 3], var[(b - BR_OPT_ARG) % 3]);
            else if (b < BR_HIER_REG) snprintf(n, z, "flame_fedbuff_scale_add/%s", dts[b - BR_SA]);
            else if (b < BR_HIER_LDS) snprintf(n, z, "flame_hier_fedbuff/reg/%s/%s", dts[(b - BR_HIER_REG) / 2], (b - BR_HIER_REG) % 2 ? "sync" : "fedbuff");
            else if (b < BR_HIER_LO) snprintf(n, z, "flame_hier_fedbuff/lds/%s/%s", dts[(b - BR_HIER_LDS) / 2], (b - BR_HIER_LDS) % 2 ? "sync" : "fedbuff");
            else if (b < BR_HIER_ARG) snprintf(n, z, "flame_hier_fedbuff/lo/%s/fedbuff", dts[b - BR_HIER_LO]);
            else if (b < BR_DYN) snprintf(n, z, "flame_hier_fedbuff_argmeta/%s/%s", dts[(b - BR_HIER_ARG) / 2], (b - BR_HIER_ARG) % 2 ? "sync" : "fedbuff");
            else if (b < BR_AGG_ARG_LO) snprintf(n, z, "flame_feddyn_round/%s", dts[b - BR_DYN]);
            else if (b < BR_HIER_ARG_LO) snprintf(n, z, "flame_agg_reduce_argmeta/lo_burst/%s", dts[b - BR_AGG_ARG_LO]);
            else if (b < BR_OPT_ARG_MULTI) snprintf(n, z, "flame_hier_fedbuff_argmeta/lo/%s/fedbuff", dts[b - BR_HIER_ARG_LO]);
            else if (b < BR_HIER_ARG_LDS) snprintf(n, z, "flame_fedopt_reduce_adapt_argmeta/multi/f32/%s", var[b - BR_OPT_ARG_MULTI]);
            else if (b < BR_CHAIN) snprintf(n, z, "flame_hier_fedbuff_argmeta/lds/%s/%s", dts[(b - BR_HIER_ARG_LDS) / 2], (b - BR_HIER_ARG_LDS) % 2 ? "sync" : "fedbuff");
            else if (b < BR_AGG_LOB) snprintf(n, z, "flame_fedopt_chain/%s/%s", dts[(b - BR_CHAIN) / 3], var[(b - BR_CHAIN) % 3]);
            else if (b < BR_EW) snprintf(n, z, "flame_agg_reduce/lo_burst/%s", dts[b - BR_AGG_LOB]);
            else if (b < BR_EW_SEG) snprintf(n, z, "flame_elementwise");
            else snprintf(n, z, "flame_elementwise_segments");
        }
        return true;
    }();
    (void)once;
    return (i >= 0 && i < BR_COUNT) ? names[i] : nullptr;
}

// check_launch + count the branch on success
int launched(int br, const char* what) {
    const int rc = check_launch(what);
    if (rc == FLAME_OK) g_launches[br].fetch_add(1, std::memory_order_relaxed);
    return rc;
}

int validate(const flame_segment* segs, int32_t n_segs, int64_t n_chunks, int32_t n_clients, const void* clients) {
    if (!segs || n_segs <= 0) return set_err(FLAME_EINVAL, "segment table is NULL or n_segs <= 0");
    if (n_chunks <= 0 || n_chunks > 0x7FFFFFFFll) return set_err(FLAME_EINVAL, "n_chunks out of range: %lld", (long long)n_chunks);
    if (n_clients < 0) return set_err(FLAME_EINVAL, "n_clients < 0");
    if (n_clients > 0 && !clients) return set_err(FLAME_EINVAL, "client pointer table is NULL");
    return FLAME_OK;
}

}  // namespace

// ==================================================================== C ABI
extern "C" {

int flame_abi_version(void) { return FLAME_ABI_VERSION; }

const char* flame_last_error(void) { return g_err; }

int64_t flame_chunk_elems(int dtype) {
    switch (dtype) {
    case FLAME_F32: return chunk_elems<FLAME_F32>();
    case FLAME_BF16: return chunk_elems<FLAME_BF16>();
    case FLAME_F16: return chunk_elems<FLAME_F16>();
    case FLAME_F64: return chunk_elems<FLAME_F64>();
    case FLAME_I64: return chunk_elems<FLAME_I64>();
    case FLAME_I32: return chunk_elems<FLAME_I32>();
    default: return 0;
    }
}

int64_t flame_scale_add_chunk_elems(int dtype) {
    switch (dtype) {
    case FLAME_F32: return kEwBlock * SA<FLAME_F32>::EPT;
    case FLAME_F64: return kEwBlock * SA<FLAME_F64>::EPT;
    case FLAME_BF16: return kEwBlock * SA<FLAME_BF16>::EPT;
    case FLAME_F16: return kEwBlock * SA<FLAME_F16>::EPT;
    default: return 0;
    }
}

int flame_agg_reduce(int dtype, unsigned flags, const flame_segment* segs, int32_t n_segs, int64_t n_chunks,
                     const void* const* clients, int32_t n_clients, const float* rates32, const double* rates64,
                     void* stream) {
    int rc = validate(segs, n_segs, n_chunks, n_clients, clients);
    if (rc) return rc;
    if ((flags & FLAME_AGG_INIT_FIRST) && n_clients < 1)
        return set_err(FLAME_EINVAL, "FLAME_AGG_INIT_FIRST needs at least one client");
    if (flags & ~(FLAME_AGG_INIT_FIRST | FLAME_AGG_SEG_RATES | FLAME_AGG_XCD_MAP))
        return set_err(FLAME_EINVAL, "flame_agg_reduce: unknown flags 0x%x", flags);
    if (dtype == FLAME_F64 ? (n_clients > 0 && !rates64) : (n_clients > 0 && !rates32))
        return set_err(FLAME_EINVAL, "rate array is NULL");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const dim3 block(kBlock);
    auto cl = reinterpret_cast<const uint64_t*>(clients);
#define FLAME_AGG_LAUNCH(DT, CUV, G, LDS, BR)                                                                   \
    hipLaunchKernelGGL((agg_reduce_kernel<DT, CUV, G>), dim3(static_cast<unsigned>((n_chunks + G - 1) / G)),    \
                       block, LDS, st, segs, n_segs, cl, n_clients, rates32, rates64, flags, n_chunks);         \
    return launched(BR, "flame_agg_reduce");
    // long-lived workgroups over many chunks: two per CU, fewer loads in flight per lane; below
    // kLoBurstMaxClients clients with their outputs held in LDS and stored in bursts
    if (n_clients >= kLoMinClients && n_chunks >= kLoMinChunks) {
        if (n_clients < kLoBurstMaxClients) {
            switch (dtype) {
            case FLAME_F32: FLAME_AGG_LAUNCH(FLAME_F32, kLoUnroll, kLoWGC, kLoDynLds, BR_AGG_LOB + FLAME_F32)
            case FLAME_BF16: FLAME_AGG_LAUNCH(FLAME_BF16, kLoUnroll16, kLoWGC, kLoDynLds, BR_AGG_LOB + FLAME_BF16)
            case FLAME_F16: FLAME_AGG_LAUNCH(FLAME_F16, kLoUnroll16, kLoWGC, kLoDynLds, BR_AGG_LOB + FLAME_F16)
            default: break;      // f64 / integers: the general launch below
            }
        }
        switch (dtype) {
        case FLAME_F32: FLAME_AGG_LAUNCH(FLAME_F32, kLoUnroll, 1, kLoLds, BR_AGG_LO + FLAME_F32)
        case FLAME_BF16: FLAME_AGG_LAUNCH(FLAME_BF16, kLoUnroll16, 1, kLoLds, BR_AGG_LO + FLAME_BF16)
        case FLAME_F16: FLAME_AGG_LAUNCH(FLAME_F16, kLoUnroll16, 1, kLoLds, BR_AGG_LO + FLAME_F16)
        default: break;      // f64 / integers: the general launch below
        }
    }
    switch (dtype) {
    case FLAME_F32: FLAME_AGG_LAUNCH(FLAME_F32, kClientUnroll, 1, 0, BR_AGG + FLAME_F32)
    case FLAME_BF16: FLAME_AGG_LAUNCH(FLAME_BF16, kClientUnroll16, 1, 0, BR_AGG + FLAME_BF16)
    case FLAME_F16: FLAME_AGG_LAUNCH(FLAME_F16, kClientUnroll16, 1, 0, BR_AGG + FLAME_F16)
    case FLAME_F64: FLAME_AGG_LAUNCH(FLAME_F64, kClientUnroll, 1, 0, BR_AGG + FLAME_F64)
    case FLAME_I64: FLAME_AGG_LAUNCH(FLAME_I64, 4, 1, 0, BR_AGG + FLAME_I64)
    case FLAME_I32: FLAME_AGG_LAUNCH(FLAME_I32, 4, 1, 0, BR_AGG + FLAME_I32)
    default:
        return set_err(FLAME_ENOTSUP, "flame_agg_reduce: unsupported dtype %d", dtype);
    }
#undef FLAME_AGG_LAUNCH
}

int flame_agg_reduce_argmeta(int dtype, unsigned flags, const void* host_meta, int64_t meta_bytes, int32_t n_segs,
                             int64_t n_chunks, int32_t n_clients, int64_t off_clients, int64_t off_r32,
                             int64_t off_r64, void* stream) {
    if (!host_meta || meta_bytes <= 0 || meta_bytes % 8 || meta_bytes > static_cast<int64_t>(sizeof(ArgMeta)))
        return set_err(FLAME_EINVAL, "flame_agg_reduce_argmeta: metadata block must be 8..%d bytes, a multiple of 8",
                       static_cast<int>(sizeof(ArgMeta)));
    if (n_segs <= 0 || n_clients < 0) return set_err(FLAME_EINVAL, "flame_agg_reduce_argmeta: n_segs <= 0 or n_clients < 0");
    if (n_chunks <= 0 || n_chunks > 0x7FFFFFFFll) return set_err(FLAME_EINVAL, "n_chunks out of range: %lld", (long long)n_chunks);
    if ((flags & FLAME_AGG_INIT_FIRST) && n_clients < 1)
        return set_err(FLAME_EINVAL, "FLAME_AGG_INIT_FIRST needs at least one client");
    if (flags & ~(FLAME_AGG_INIT_FIRST | FLAME_AGG_SEG_RATES | FLAME_AGG_XCD_MAP))
        return set_err(FLAME_EINVAL, "flame_agg_reduce_argmeta: unknown flags 0x%x", flags);
    const int64_t rows = (flags & FLAME_AGG_SEG_RATES) ? n_segs : 1;
    auto inside = [&](int64_t off, int64_t bytes) { return off >= 0 && off % 8 == 0 && off + bytes <= meta_bytes; };
    if (static_cast<int64_t>(n_segs) * static_cast<int64_t>(sizeof(flame_segment)) > meta_bytes ||
        !inside(off_clients, static_cast<int64_t>(n_segs) * n_clients * 8))
        return set_err(FLAME_EINVAL, "flame_agg_reduce_argmeta: segment / client table outside the metadata block");
    const bool f64 = dtype == FLAME_F64;
    if (n_clients > 0 && (f64 ? !inside(off_r64, rows * n_clients * 8) : !inside(off_r32, rows * n_clients * 4)))
        return set_err(FLAME_EINVAL, "flame_agg_reduce_argmeta: rate array outside the metadata block");
    ArgMeta m;
    std::memcpy(m.w, host_meta, static_cast<size_t>(meta_bytes));
    const int oc = static_cast<int>(off_clients / 8);
    const int o32 = (!f64 && n_clients > 0) ? static_cast<int>(off_r32 / 8) : -1;
    const int o64 = (f64 && n_clients > 0) ? static_cast<int>(off_r64 / 8) : -1;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const dim3 grid(static_cast<unsigned>(n_chunks)), block(kBlock);
#define FLAME_ARGMETA_LAUNCH(DT, CUV) \
    hipLaunchKernelGGL((agg_reduce_kernel_argmeta<DT, CUV, 1>), grid, block, 0, st, m, n_segs, n_clients, \
                       oc, o32, o64, flags, n_chunks)
    // a long launch with few segments (its table fits the kernel arguments): the same low-residency
    // instantiation as flame_agg_reduce's
    if (n_clients >= kLoMinClients && n_chunks >= kLoMinChunks &&
        (dtype == FLAME_F32 || dtype == FLAME_BF16 || dtype == FLAME_F16)) {
#define FLAME_ARGMETA_LO(DT, CUV, G, LDS)                                                                      \
        hipLaunchKernelGGL((agg_reduce_kernel_argmeta<DT, CUV, G>), dim3(static_cast<unsigned>((n_chunks + G - 1) / G)), \
                           block, LDS, st, m, n_segs, n_clients, oc, o32, o64, flags, n_chunks)
        static_assert((kArgMetaWords - 10) < kLoBurstMaxClients,
                      "a kernel-argument launch can hold kLoBurstMaxClients clients: it needs the plain instantiation too");
        if (dtype == FLAME_F32) FLAME_ARGMETA_LO(FLAME_F32, kLoUnroll, kLoWGC, kLoDynLds);
        else if (dtype == FLAME_BF16) FLAME_ARGMETA_LO(FLAME_BF16, kLoUnroll16, kLoWGC, kLoDynLds);
        else FLAME_ARGMETA_LO(FLAME_F16, kLoUnroll16, kLoWGC, kLoDynLds);
#undef FLAME_ARGMETA_LO
        return launched(BR_AGG_ARG_LO + dtype, "flame_agg_reduce_argmeta");
    }
    switch (dtype) {
    case FLAME_F32: FLAME_ARGMETA_LAUNCH(FLAME_F32, kClientUnroll); break;
    case FLAME_BF16: FLAME_ARGMETA_LAUNCH(FLAME_BF16, kClientUnroll16); break;
    case FLAME_F16: FLAME_ARGMETA_LAUNCH(FLAME_F16, kClientUnroll16); break;
    case FLAME_F64: FLAME_ARGMETA_LAUNCH(FLAME_F64, kClientUnroll); break;
    case FLAME_I64: FLAME_ARGMETA_LAUNCH(FLAME_I64, 4); break;
    case FLAME_I32: FLAME_ARGMETA_LAUNCH(FLAME_I32, 4); break;
    default:
        return set_err(FLAME_ENOTSUP, "flame_agg_reduce_argmeta: unsupported dtype %d", dtype);
    }
#undef FLAME_ARGMETA_LAUNCH
    return launched(BR_AGG_ARG + dtype, "flame_agg_reduce_argmeta");
}

int64_t flame_agg_argmeta_max_bytes(void) { return static_cast<int64_t>(sizeof(ArgMeta)); }

int flame_fedopt_reduce_adapt(int dtype, int variant, unsigned flags, const flame_segment* segs, int32_t n_segs,
                              int64_t n_chunks, const void* const* clients, int32_t n_clients,
                              const float* rates32, float b1, float omb1, float b2, float omb2, float eta,
                              float tau, void* stream) {
    int rc = validate(segs, n_segs, n_chunks, n_clients, clients);
    if (rc) return rc;
    if (n_clients > 0 && !rates32) return set_err(FLAME_EINVAL, "rate array is NULL");
    if (variant < FLAME_FEDADAM || variant > FLAME_FEDADAGRAD)
        return set_err(FLAME_ENOTSUP, "flame_fedopt_reduce_adapt: unknown variant %d", variant);
    if (flags & ~(FLAME_OPT_STATE_ZERO | FLAME_OPT_XCD_MAP))
        return set_err(FLAME_EINVAL, "flame_fedopt_reduce_adapt: unknown flags 0x%x", flags);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    // kOptWGC chunks per workgroup (outputs held in LDS) for fp32 launches big enough to fill
    // the GPU several times over; one chunk per workgroup otherwise
    const bool multi = dtype == FLAME_F32 && n_chunks >= 8ll * 256 * kOptWGC;
    const dim3 grid(static_cast<unsigned>(multi ? (n_chunks + kOptWGC - 1) / kOptWGC : n_chunks)), block(kBlock);
    auto cl = reinterpret_cast<const uint64_t*>(clients);
#define FLAME_OPT_LAUNCH1(DT, CUV, G)                                                                          \
    switch (variant) {                                                                                         \
    case FLAME_FEDADAM:                                                                                        \
        hipLaunchKernelGGL((fedopt_kernel<DT, FLAME_FEDADAM, CUV, G>), grid, block, 0, st, segs, n_segs, cl,    \
                           n_clients, rates32, flags, b1, omb1, b2, omb2, eta, tau, n_chunks);                 \
        break;                                                                                                 \
    case FLAME_FEDYOGI:                                                                                        \
        hipLaunchKernelGGL((fedopt_kernel<DT, FLAME_FEDYOGI, CUV, G>), grid, block, 0, st, segs, n_segs, cl,    \
                           n_clients, rates32, flags, b1, omb1, b2, omb2, eta, tau, n_chunks);                 \
        break;                                                                                                 \
    default:                                                                                                   \
        hipLaunchKernelGGL((fedopt_kernel<DT, FLAME_FEDADAGRAD, CUV, G>), grid, block, 0, st, segs, n_segs, cl, \
                           n_clients, rates32, flags, b1, omb1, b2, omb2, eta, tau, n_chunks);                 \
        break;                                                                                                 \
    }
    switch (dtype) {
    case FLAME_F32:
        if (multi) { FLAME_OPT_LAUNCH1(FLAME_F32, kOptUnroll, kOptWGC) }
        else { FLAME_OPT_LAUNCH1(FLAME_F32, kClientUnroll, 1) }
        break;
    case FLAME_BF16: FLAME_OPT_LAUNCH1(FLAME_BF16, kClientUnroll16, 1) break;
    case FLAME_F16: FLAME_OPT_LAUNCH1(FLAME_F16, kClientUnroll16, 1) break;
    default:
        return set_err(FLAME_ENOTSUP, "flame_fedopt_reduce_adapt: dtype %d not supported (f32, bf16, f16)", dtype);
    }
#undef FLAME_OPT_LAUNCH1
    return launched(multi ? BR_OPT_MULTI + variant : BR_OPT + dtype * 3 + variant, "flame_fedopt_reduce_adapt");
}

int flame_fedopt_chain(int dtype, int variant, unsigned flags, const flame_segment* segs, int32_t n_segs,
                       int64_t n_chunks, const void* const* clients, int32_t n_clients, const float* rates32,
                       const uint8_t* step_end, float b1, float omb1, float b2, float omb2, float eta, float tau,
                       void* stream) {
    int rc = validate(segs, n_segs, n_chunks, n_clients, clients);
    if (rc) return rc;
    if (n_clients < 1 || !rates32 || !step_end)
        return set_err(FLAME_EINVAL, "flame_fedopt_chain: needs >= 1 client, a rate array and a step_end array");
    if (variant < FLAME_FEDADAM || variant > FLAME_FEDADAGRAD)
        return set_err(FLAME_ENOTSUP, "flame_fedopt_chain: unknown variant %d", variant);
    if (flags & ~FLAME_OPT_STATE_ZERO) return set_err(FLAME_EINVAL, "flame_fedopt_chain: unknown flags 0x%x", flags);
    if (dtype != FLAME_F32 && dtype != FLAME_BF16 && dtype != FLAME_F16)
        return set_err(FLAME_ENOTSUP, "flame_fedopt_chain: dtype %d not supported (f32, bf16, f16)", dtype);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const dim3 grid(static_cast<unsigned>(n_chunks)), block(kBlock);
    auto cl = reinterpret_cast<const uint64_t*>(clients);
#define FLAME_CHAIN_LAUNCH(DT, V, CUV)                                                                              \
    hipLaunchKernelGGL((fedopt_chain_kernel<DT, V, CUV>), grid, block, DT == FLAME_F32 ? kChainLds : 0, st, segs,   \
                       n_segs, cl, n_clients,                                                                       \
                       rates32,                                                                                     \
                       step_end, flags, b1, omb1, b2, omb2, eta, tau)
#define FLAME_CHAIN_VARIANTS(DT, CUV)                                                  \
    if (variant == FLAME_FEDADAM) FLAME_CHAIN_LAUNCH(DT, FLAME_FEDADAM, CUV);          \
    else if (variant == FLAME_FEDYOGI) FLAME_CHAIN_LAUNCH(DT, FLAME_FEDYOGI, CUV);     \
    else FLAME_CHAIN_LAUNCH(DT, FLAME_FEDADAGRAD, CUV);
    if (dtype == FLAME_F32) { FLAME_CHAIN_VARIANTS(FLAME_F32, kChainUnroll) }
    else if (dtype == FLAME_BF16) { FLAME_CHAIN_VARIANTS(FLAME_BF16, kChainUnroll16) }
    else { FLAME_CHAIN_VARIANTS(FLAME_F16, kChainUnroll16) }
#undef FLAME_CHAIN_VARIANTS
#undef FLAME_CHAIN_LAUNCH
    return launched(BR_CHAIN + dtype * 3 + variant, "flame_fedopt_chain");
}

int flame_fedopt_reduce_adapt_argmeta(int dtype, int variant, unsigned flags, const void* host_meta,
                                      int64_t meta_bytes, int32_t n_segs, int64_t n_chunks, int32_t n_clients,
                                      int64_t off_clients, int64_t off_r32, float b1, float omb1, float b2,
                                      float omb2, float eta, float tau, void* stream) {
    if (!host_meta || meta_bytes <= 0 || meta_bytes % 8 || meta_bytes > static_cast<int64_t>(sizeof(ArgMeta)))
        return set_err(FLAME_EINVAL, "flame_fedopt_reduce_adapt_argmeta: metadata block must be 8..%d bytes, a multiple of 8",
                       static_cast<int>(sizeof(ArgMeta)));
    if (n_segs <= 0 || n_clients < 0)
        return set_err(FLAME_EINVAL, "flame_fedopt_reduce_adapt_argmeta: n_segs <= 0 or n_clients < 0");
    if (n_chunks <= 0 || n_chunks > 0x7FFFFFFFll) return set_err(FLAME_EINVAL, "n_chunks out of range: %lld", (long long)n_chunks);
    if (flags & ~(FLAME_OPT_STATE_ZERO | FLAME_OPT_XCD_MAP))
        return set_err(FLAME_EINVAL, "flame_fedopt_reduce_adapt_argmeta: unknown flags 0x%x", flags);
    if (variant < FLAME_FEDADAM || variant > FLAME_FEDADAGRAD)
        return set_err(FLAME_ENOTSUP, "flame_fedopt_reduce_adapt_argmeta: unknown variant %d", variant);
    auto inside = [&](int64_t off, int64_t bytes) { return off >= 0 && off % 8 == 0 && off + bytes <= meta_bytes; };
    if (static_cast<int64_t>(n_segs) * static_cast<int64_t>(sizeof(flame_segment)) > meta_bytes ||
        !inside(off_clients, static_cast<int64_t>(n_segs) * n_clients * 8) ||
        (n_clients > 0 && !inside(off_r32, static_cast<int64_t>(n_clients) * 4)))
        return set_err(FLAME_EINVAL, "flame_fedopt_reduce_adapt_argmeta: a table lies outside the metadata block");
    ArgMeta m;
    std::memcpy(m.w, host_meta, static_cast<size_t>(meta_bytes));
    const int oc = static_cast<int>(off_clients / 8);
    const int o32 = n_clients > 0 ? static_cast<int>(off_r32 / 8) : -1;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    // the instantiation flame_fedopt_reduce_adapt picks for the same launch
    const bool multi = dtype == FLAME_F32 && n_chunks >= 8ll * 256 * kOptWGC;
    const dim3 grid(static_cast<unsigned>(multi ? (n_chunks + kOptWGC - 1) / kOptWGC : n_chunks)), block(kBlock);
#define FLAME_OPT_ARGMETA_LAUNCH(DT, CUV, G)                                                                     \
    switch (variant) {                                                                                           \
    case FLAME_FEDADAM:                                                                                          \
        hipLaunchKernelGGL((fedopt_kernel_argmeta<DT, FLAME_FEDADAM, CUV, G>), grid, block, 0, st, m, n_segs,     \
                           n_clients, oc, o32, flags, b1, omb1, b2, omb2, eta, tau, n_chunks);                   \
        break;                                                                                                   \
    case FLAME_FEDYOGI:                                                                                          \
        hipLaunchKernelGGL((fedopt_kernel_argmeta<DT, FLAME_FEDYOGI, CUV, G>), grid, block, 0, st, m, n_segs,     \
                           n_clients, oc, o32, flags, b1, omb1, b2, omb2, eta, tau, n_chunks);                   \
        break;                                                                                                   \
    default:                                                                                                     \
        hipLaunchKernelGGL((fedopt_kernel_argmeta<DT, FLAME_FEDADAGRAD, CUV, G>), grid, block, 0, st, m, n_segs,  \
                           n_clients, oc, o32, flags, b1, omb1, b2, omb2, eta, tau, n_chunks);                   \
        break;                                                                                                   \
    }
    switch (dtype) {
    case FLAME_F32:
        if (multi) { FLAME_OPT_ARGMETA_LAUNCH(FLAME_F32, kOptUnroll, kOptWGC) }
        else { FLAME_OPT_ARGMETA_LAUNCH(FLAME_F32, kClientUnroll, 1) }
        break;
    case FLAME_BF16: FLAME_OPT_ARGMETA_LAUNCH(FLAME_BF16, kClientUnroll16, 1) break;
    case FLAME_F16: FLAME_OPT_ARGMETA_LAUNCH(FLAME_F16, kClientUnroll16, 1) break;
    default:
        return set_err(FLAME_ENOTSUP, "flame_fedopt_reduce_adapt_argmeta: dtype %d not supported (f32, bf16, f16)", dtype);
    }
#undef FLAME_OPT_ARGMETA_LAUNCH
    if (multi) return launched(BR_OPT_ARG_MULTI + variant, "flame_fedopt_reduce_adapt_argmeta");
    return launched(BR_OPT_ARG + dtype * 3 + variant, "flame_fedopt_reduce_adapt_argmeta");
}

int flame_fedbuff_scale_add(int dtype, const flame_segment* segs, int32_t n_segs, int64_t n_chunks, int64_t goal,
                            void* stream) {
    int rc = validate(segs, n_segs, n_chunks, 0, nullptr);
    if (rc) return rc;
    if (goal == 0) return set_err(FLAME_EINVAL, "agg_goal must be nonzero");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const dim3 grid(static_cast<unsigned>(n_chunks)), block(kEwBlock);
    const float gf = static_cast<float>(goal);
    const double gd = static_cast<double>(goal);
    switch (dtype) {
    case FLAME_F32: hipLaunchKernelGGL((scale_add_kernel<FLAME_F32>), grid, block, 0, st, segs, n_segs, gf, gd); break;
    case FLAME_F64: hipLaunchKernelGGL((scale_add_kernel<FLAME_F64>), grid, block, 0, st, segs, n_segs, gf, gd); break;
    case FLAME_BF16: hipLaunchKernelGGL((scale_add_kernel<FLAME_BF16>), grid, block, 0, st, segs, n_segs, gf, gd); break;
    case FLAME_F16: hipLaunchKernelGGL((scale_add_kernel<FLAME_F16>), grid, block, 0, st, segs, n_segs, gf, gd); break;
    default:
        return set_err(FLAME_ENOTSUP, "flame_fedbuff_scale_add: dtype %d not supported (integer tensors raise in the reference)", dtype);
    }
    return launched(BR_SA + dtype, "flame_fedbuff_scale_add");
}

int flame_hier_fedbuff(int dtype, unsigned flags, const flame_hier_segment* segs, int32_t n_segs, int64_t n_chunks,
                       int32_t n_mids, int32_t n_clients, const void* const* mid_w, const void* const* mid_delta,
                       const void* const* clients, const float* mid_rates, const float* mid_goal,
                       const float* top_rates, float top_goal, void* stream) {
    if (!segs || n_segs <= 0) return set_err(FLAME_EINVAL, "segment table is NULL or n_segs <= 0");
    if (n_chunks <= 0 || n_chunks > 0x7FFFFFFFll) return set_err(FLAME_EINVAL, "n_chunks out of range: %lld", (long long)n_chunks);
    if (n_mids < 1 || n_clients < 1) return set_err(FLAME_EINVAL, "flame_hier_fedbuff: need >= 1 middle and >= 1 arrival per middle");
    if (!mid_w || !clients || !mid_rates || !mid_goal || !top_rates)
        return set_err(FLAME_EINVAL, "flame_hier_fedbuff: NULL table");
    if (flags & ~(FLAME_HIER_TOP_ACCUM | FLAME_HIER_TOP_APPLY | FLAME_HIER_MID_READONLY | FLAME_HIER_SYNC))
        return set_err(FLAME_EINVAL, "flame_hier_fedbuff: unknown flags 0x%x", flags);
    if ((flags & FLAME_HIER_SYNC) && ((flags & FLAME_HIER_TOP_APPLY) || !(flags & FLAME_HIER_TOP_ACCUM)))
        return set_err(FLAME_EINVAL, "flame_hier_fedbuff: FLAME_HIER_SYNC needs FLAME_HIER_TOP_ACCUM (the top's "
                                     "FedAvg starts from its weights) and no FLAME_HIER_TOP_APPLY");
    if ((flags & FLAME_HIER_TOP_APPLY) && top_goal == 0.f) return set_err(FLAME_EINVAL, "top agg_goal must be nonzero");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const dim3 grid(static_cast<unsigned>(n_chunks)), block(kBlock);
    auto w = reinterpret_cast<const uint64_t*>(mid_w);
    auto d = reinterpret_cast<const uint64_t*>(mid_delta);
    auto cl = reinterpret_cast<const uint64_t*>(clients);
    const bool sync = (flags & FLAME_HIER_SYNC) != 0;
    // many middles (config 5: 64 per GPU): LDS-held store groups.  One middle over a long launch
    // (a FedBuff aggregator's fused scale_add / a middle's scale_add + delta over >= 64 queued
    // arrivals): fewer workgroups per CU, fewer loads in flight -- fp32 2 per CU, 16-bit 3 per CU,
    // unroll 3 (64 x 25M: 1.058 -> 0.989 ms fp32, 0.533 -> 0.509 ms bf16; tools/fedbuff_sweep.py,
    // profiles/r03zv_fedbuff_*.log).  Otherwise (small hierarchies): register groups, full residency.
    const bool lds = n_mids >= kHLdsMinMids;
    const bool lo = !lds && !sync && n_mids == 1 && n_clients >= kHLoMinClients && n_chunks >= kHLoMinChunks;
#define FLAME_HIER_GO(DT, CUV, SY, HB, HL, LDSB)                                                              \
    hipLaunchKernelGGL((hier_fedbuff_kernel<DT, CUV, SY, HB, HL>), grid, block, LDSB, st, segs, n_segs, n_mids, \
                       n_clients, w, d, cl, mid_rates, mid_goal, top_rates, top_goal, flags)
#define FLAME_HIER_LAUNCH(DT, CUV, CUL, LOLDS)                                                                  \
    if (lds) {                                                                                                 \
        if (sync) FLAME_HIER_GO(DT, CUL, true, kHBL, true, 0);                                                 \
        else FLAME_HIER_GO(DT, CUL, false, kHBL, true, 0);                                                     \
        br = BR_HIER_LDS + DT * 2 + sync;                                                                      \
    } else if (lo) {                                                                                           \
        FLAME_HIER_GO(DT, kHLoUnroll, false, kHB, false, LOLDS);                                               \
        br = BR_HIER_LO + DT;                                                                                  \
    } else {                                                                                                   \
        if (sync) FLAME_HIER_GO(DT, CUV, true, kHB, false, 0);                                                 \
        else FLAME_HIER_GO(DT, CUV, false, kHB, false, 0);                                                     \
        br = BR_HIER_REG + DT * 2 + sync;                                                                      \
    }
    int br = 0;
    switch (dtype) {
    case FLAME_F32: FLAME_HIER_LAUNCH(FLAME_F32, kClientUnroll, kClientUnroll, kHLoLdsF32) break;
    case FLAME_BF16: FLAME_HIER_LAUNCH(FLAME_BF16, kHierUnroll16, kHierLdsUnroll16, kHLoLds16) break;
    case FLAME_F16: FLAME_HIER_LAUNCH(FLAME_F16, kHierUnroll16, kHierLdsUnroll16, kHLoLds16) break;
#undef FLAME_HIER_GO
#undef FLAME_HIER_LAUNCH
    default:
        return set_err(FLAME_ENOTSUP, "flame_hier_fedbuff: dtype %d not supported (f32, bf16, f16)", dtype);
    }
    return launched(br, "flame_hier_fedbuff");
}

int flame_hier_fedbuff_argmeta(int dtype, unsigned flags, const void* host_meta, int64_t meta_bytes, int32_t n_segs,
                               int64_t n_chunks, int32_t n_mids, int32_t n_clients, int64_t off_mid_w,
                               int64_t off_mid_delta, int64_t off_clients, int64_t off_mid_rates,
                               int64_t off_mid_goal, int64_t off_top_rates, float top_goal, void* stream) {
    if (!host_meta || meta_bytes <= 0 || meta_bytes % 8 || meta_bytes > static_cast<int64_t>(sizeof(ArgMeta)))
        return set_err(FLAME_EINVAL, "flame_hier_fedbuff_argmeta: metadata block must be 8..%d bytes, a multiple of 8",
                       static_cast<int>(sizeof(ArgMeta)));
    if (n_segs <= 0) return set_err(FLAME_EINVAL, "segment table is empty");
    if (n_chunks <= 0 || n_chunks > 0x7FFFFFFFll) return set_err(FLAME_EINVAL, "n_chunks out of range: %lld", (long long)n_chunks);
    if (n_mids < 1 || n_clients < 1) return set_err(FLAME_EINVAL, "flame_hier_fedbuff_argmeta: need >= 1 middle and >= 1 arrival per middle");
    if (flags & ~(FLAME_HIER_TOP_ACCUM | FLAME_HIER_TOP_APPLY | FLAME_HIER_MID_READONLY | FLAME_HIER_SYNC))
        return set_err(FLAME_EINVAL, "flame_hier_fedbuff_argmeta: unknown flags 0x%x", flags);
    if ((flags & FLAME_HIER_SYNC) && ((flags & FLAME_HIER_TOP_APPLY) || !(flags & FLAME_HIER_TOP_ACCUM)))
        return set_err(FLAME_EINVAL, "flame_hier_fedbuff_argmeta: FLAME_HIER_SYNC needs FLAME_HIER_TOP_ACCUM and no FLAME_HIER_TOP_APPLY");
    if ((flags & FLAME_HIER_TOP_APPLY) && top_goal == 0.f) return set_err(FLAME_EINVAL, "top agg_goal must be nonzero");
    auto inside = [&](int64_t off, int64_t bytes) { return off >= 0 && off % 8 == 0 && off + bytes <= meta_bytes; };
    const int64_t S = n_segs, M = n_mids, C = n_clients;
    if (S * static_cast<int64_t>(sizeof(flame_hier_segment)) > meta_bytes || !inside(off_mid_w, S * M * 8) ||
        (off_mid_delta >= 0 && !inside(off_mid_delta, S * M * 8)) || !inside(off_clients, S * M * C * 8) ||
        !inside(off_mid_rates, M * C * 4) || !inside(off_mid_goal, M * 4) || !inside(off_top_rates, M * 4))
        return set_err(FLAME_EINVAL, "flame_hier_fedbuff_argmeta: a table lies outside the metadata block");
    ArgMeta m;
    std::memcpy(m.w, host_meta, static_cast<size_t>(meta_bytes));
    const int ow = static_cast<int>(off_mid_w / 8), od = off_mid_delta >= 0 ? static_cast<int>(off_mid_delta / 8) : -1;
    const int oc = static_cast<int>(off_clients / 8), orr = static_cast<int>(off_mid_rates / 8);
    const int og = static_cast<int>(off_mid_goal / 8), ot = static_cast<int>(off_top_rates / 8);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const dim3 grid(static_cast<unsigned>(n_chunks)), block(kBlock);
    const bool sync = (flags & FLAME_HIER_SYNC) != 0;
    // the instantiation flame_hier_fedbuff picks for the same launch shape: LDS store groups for
    // many middles, the low-residency one for one middle over a long launch (a FedBuff
    // aggregator's fused scale_add of >= 64 arrivals into a model of a few keys), else register groups
    const bool lds = n_mids >= kHLdsMinMids;
    const bool lo = !lds && !sync && n_mids == 1 && n_clients >= kHLoMinClients && n_chunks >= kHLoMinChunks;
#define FLAME_HIER_ARG_GO(DT, CUV, SY, HB, HL, LDSB)                                                            \
    hipLaunchKernelGGL((hier_fedbuff_kernel_argmeta<DT, CUV, SY, HB, HL>), grid, block, LDSB, st, m, n_segs, n_mids, \
                       n_clients, ow, od, oc, orr, og, ot, top_goal, flags)
#define FLAME_HIER_ARG_LAUNCH(DT, CUV, CUL, LOLDS)                                                              \
    if (lds) {                                                                                                 \
        if (sync) FLAME_HIER_ARG_GO(DT, CUL, true, kHBL, true, 0);                                             \
        else FLAME_HIER_ARG_GO(DT, CUL, false, kHBL, true, 0);                                                 \
        br = BR_HIER_ARG_LDS + DT * 2 + sync;                                                                  \
    } else if (lo) {                                                                                           \
        FLAME_HIER_ARG_GO(DT, kHLoUnroll, false, kHB, false, LOLDS);                                           \
        br = BR_HIER_ARG_LO + DT;                                                                              \
    } else {                                                                                                   \
        if (sync) FLAME_HIER_ARG_GO(DT, CUV, true, kHB, false, 0);                                             \
        else FLAME_HIER_ARG_GO(DT, CUV, false, kHB, false, 0);                                                 \
        br = BR_HIER_ARG + DT * 2 + sync;                                                                      \
    }
    int br = 0;
    switch (dtype) {
    case FLAME_F32: FLAME_HIER_ARG_LAUNCH(FLAME_F32, kClientUnroll, kClientUnroll, kHLoLdsF32) break;
    case FLAME_BF16: FLAME_HIER_ARG_LAUNCH(FLAME_BF16, kHierUnroll16, kHierLdsUnroll16, kHLoLds16) break;
    case FLAME_F16: FLAME_HIER_ARG_LAUNCH(FLAME_F16, kHierUnroll16, kHierLdsUnroll16, kHLoLds16) break;
#undef FLAME_HIER_ARG_GO
#undef FLAME_HIER_ARG_LAUNCH
    default:
        return set_err(FLAME_ENOTSUP, "flame_hier_fedbuff_argmeta: dtype %d not supported (f32, bf16, f16)", dtype);
    }
    return launched(br, "flame_hier_fedbuff_argmeta");
}

int flame_hier_resident_per_cu(int dtype, unsigned flags, int32_t n_mids) {
    if (n_mids < 1) return -set_err(FLAME_EINVAL, "flame_hier_resident_per_cu: n_mids < 1");
    const bool sync = (flags & FLAME_HIER_SYNC) != 0;
    const bool lds = n_mids >= kHLdsMinMids;
    const void* f = nullptr;
    // the instantiation flame_hier_fedbuff picks for these arguments (the one-middle low-residency
    // launch aside, which depends on the launch size)
#define FLAME_HIER_PICK(DT, CUV, CUL)                                                                          \
    if (lds) f = sync ? reinterpret_cast<const void*>(hier_fedbuff_kernel<DT, CUL, true, kHBL, true>)          \
                      : reinterpret_cast<const void*>(hier_fedbuff_kernel<DT, CUL, false, kHBL, true>);        \
    else f = sync ? reinterpret_cast<const void*>(hier_fedbuff_kernel<DT, CUV, true, kHB, false>)              \
                  : reinterpret_cast<const void*>(hier_fedbuff_kernel<DT, CUV, false, kHB, false>);
    switch (dtype) {
    case FLAME_F32: FLAME_HIER_PICK(FLAME_F32, kClientUnroll, kClientUnroll) break;
    case FLAME_BF16: FLAME_HIER_PICK(FLAME_BF16, kHierUnroll16, kHierLdsUnroll16) break;
    case FLAME_F16: FLAME_HIER_PICK(FLAME_F16, kHierUnroll16, kHierLdsUnroll16) break;
#undef FLAME_HIER_PICK
    default:
        return -set_err(FLAME_ENOTSUP, "flame_hier_resident_per_cu: dtype %d not supported (f32, bf16, f16)", dtype);
    }
    int blocks = 0;
    const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, f, kBlock, 0);
    if (e != hipSuccess) return -set_err(FLAME_EHIP, "hipOccupancyMaxActiveBlocksPerMultiprocessor: %s", hipGetErrorString(e));
    return blocks < 1 ? 1 : blocks;
}

int flame_feddyn_round(int dtype, const flame_dyn_segment* segs, int32_t n_segs, int64_t n_chunks,
                       const void* const* steps, const uint32_t* step_flags, int32_t n_steps, int32_t n_phase1,
                       double rate_avg, double rate_mean, void* stream) {
    if (!segs || n_segs <= 0) return set_err(FLAME_EINVAL, "segment table is NULL or n_segs <= 0");
    if (n_chunks <= 0 || n_chunks > 0x7FFFFFFFll) return set_err(FLAME_EINVAL, "n_chunks out of range: %lld", (long long)n_chunks);
    if (n_steps < 1 || !steps) return set_err(FLAME_EINVAL, "flame_feddyn_round: empty step program");
    if (n_steps > 0 && !step_flags) return set_err(FLAME_EINVAL, "flame_feddyn_round: step flag array is NULL");
    if (n_phase1 < 0 || n_phase1 > n_steps)
        return set_err(FLAME_EINVAL, "flame_feddyn_round: n_phase1 %d outside [0, %d]", n_phase1, n_steps);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const dim3 grid(static_cast<unsigned>(n_chunks)), block(kBlock);
    auto sp = reinterpret_cast<const uint64_t*>(steps);
    // torch rounds the Python-float rates to the tensor's opmath type: fp32, fp64 for f64 tensors
    const float ra32 = static_cast<float>(rate_avg), rm32 = static_cast<float>(rate_mean);
    switch (dtype) {
    case FLAME_F32:
        hipLaunchKernelGGL((feddyn_kernel<FLAME_F32, kDynUnroll>), grid, block, 0, st, segs, n_segs, sp, step_flags, n_steps,
                           n_phase1, ra32, rm32, rate_avg, rate_mean);
        break;
    case FLAME_BF16:
        hipLaunchKernelGGL((feddyn_kernel<FLAME_BF16, kDynUnroll>), grid, block, 0, st, segs, n_segs, sp, step_flags, n_steps,
                           n_phase1, ra32, rm32, rate_avg, rate_mean);
        break;
    case FLAME_F16:
        hipLaunchKernelGGL((feddyn_kernel<FLAME_F16, kDynUnroll>), grid, block, 0, st, segs, n_segs, sp, step_flags, n_steps,
                           n_phase1, ra32, rm32, rate_avg, rate_mean);
        break;
    case FLAME_F64:
        hipLaunchKernelGGL((feddyn_kernel<FLAME_F64, kDynUnroll>), grid, block, 0, st, segs, n_segs, sp, step_flags, n_steps,
                           n_phase1, ra32, rm32, rate_avg, rate_mean);
        break;
    default:
        return set_err(FLAME_ENOTSUP, "flame_feddyn_round: dtype %d not supported (f32, bf16, f16, f64)", dtype);
    }
    return launched(BR_DYN + dtype, "flame_feddyn_round");
}

int flame_host_register(void* host, uint64_t nbytes) {
    if (!host || nbytes == 0) return set_err(FLAME_EINVAL, "flame_host_register: empty range");
    hipError_t e = hipHostRegister(host, static_cast<size_t>(nbytes), hipHostRegisterMapped | hipHostRegisterPortable);
    if (e != hipSuccess) return set_err(FLAME_EHIP, "hipHostRegister: %s", hipGetErrorString(e));
    return FLAME_OK;
}

int flame_host_unregister(void* host) {
    if (!host) return set_err(FLAME_EINVAL, "flame_host_unregister: NULL");
    hipError_t e = hipHostUnregister(host);
    if (e != hipSuccess) return set_err(FLAME_EHIP, "hipHostUnregister: %s", hipGetErrorString(e));
    return FLAME_OK;
}

int flame_host_device_pointer(void* host, void** device) {
    if (!host || !device) return set_err(FLAME_EINVAL, "flame_host_device_pointer: NULL");
    hipError_t e = hipHostGetDevicePointer(device, host, 0);
    if (e != hipSuccess) return set_err(FLAME_EHIP, "hipHostGetDevicePointer: %s", hipGetErrorString(e));
    return FLAME_OK;
}

int flame_synth_fill(int dtype, void* out, int64_t numel, uint64_t seed, uint64_t stream_id, int64_t start,
                     float scale, void* stream) {
    if (numel < 0 || (numel > 0 && !out)) return set_err(FLAME_EINVAL, "flame_synth_fill: bad buffer");
    if (numel == 0) return FLAME_OK;
    const uint64_t ck = mix64((seed * 0x9E3779B97F4A7C15ull) ^ ((stream_id + 1ull) * 0xD1B54A32D192ED03ull));
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    int64_t blocks = (numel + kEwBlock - 1) / kEwBlock;
    if (blocks > 8192) blocks = 8192;
    const dim3 grid(static_cast<unsigned>(blocks)), block(kEwBlock);
    switch (dtype) {
    case FLAME_F32: hipLaunchKernelGGL(synth_kernel<FLAME_F32>, grid, block, 0, st, out, numel, ck, start, scale); break;
    case FLAME_BF16: hipLaunchKernelGGL(synth_kernel<FLAME_BF16>, grid, block, 0, st, out, numel, ck, start, scale); break;
    case FLAME_F16: hipLaunchKernelGGL(synth_kernel<FLAME_F16>, grid, block, 0, st, out, numel, ck, start, scale); break;
    default: return set_err(FLAME_ENOTSUP, "flame_synth_fill: dtype %d not supported", dtype);
    }
    return check_launch("flame_synth_fill");
}

static int ew_check(const flame_ew_op* prog, int32_t n_ops, void* const* bufs, int32_t n_bufs, int64_t numel);

int flame_elementwise(const flame_ew_op* prog, int32_t n_ops, void* const* bufs, int32_t n_bufs, int64_t numel,
                      void* stream) {
    if (n_bufs < 0 || n_bufs > FLAME_EW_MAX_BUFS || (n_bufs > 0 && !bufs))
        return set_err(FLAME_EINVAL, "flame_elementwise: n_bufs %d outside [0, %d] or NULL table", n_bufs, FLAME_EW_MAX_BUFS);
    const int rc = ew_check(prog, n_ops, bufs, n_bufs, numel);
    if (rc != FLAME_OK) return rc;
    if (numel == 0 || n_ops == 0) return FLAME_OK;
    EwArgs a{};
    for (int32_t k = 0; k < n_ops; ++k) a.ops[k] = prog[k];
    for (int32_t k = 0; k < n_bufs; ++k) a.bufs[k] = bufs[k];
    a.numel = numel;
    a.n_ops = n_ops;
    int64_t blocks = (numel + kEwBlock - 1) / kEwBlock;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(ew_kernel, dim3(static_cast<unsigned>(blocks)), dim3(kEwBlock), 0,
                       reinterpret_cast<hipStream_t>(stream), a);
    return launched(BR_EW, "flame_elementwise");
}

int flame_elementwise_segments(const flame_ew_op* prog, int32_t n_ops, void* const* table, int32_t n_bufs,
                               const int64_t* seg_end, int32_t n_segs, int64_t numel, void* stream) {
    if (n_bufs < 0 || n_bufs > FLAME_EW_MAX_BUFS)
        return set_err(FLAME_EINVAL, "flame_elementwise_segments: n_bufs %d outside [0, %d]", n_bufs, FLAME_EW_MAX_BUFS);
    if (n_segs <= 0 || !table || !seg_end)
        return set_err(FLAME_EINVAL, "flame_elementwise_segments: n_segs <= 0 or a NULL table");
    const int rc = ew_check(prog, n_ops, nullptr, n_bufs, numel);      // the buffers live on the device
    if (rc != FLAME_OK) return rc;
    if (numel == 0 || n_ops == 0) return FLAME_OK;
    EwArgs a{};
    for (int32_t k = 0; k < n_ops; ++k) a.ops[k] = prog[k];
    a.table = table;
    a.seg_end = seg_end;
    a.numel = numel;
    a.n_ops = n_ops;
    a.n_segs = n_segs;
    a.n_bufs = n_bufs;
    int64_t blocks = (numel + kEwBlock - 1) / kEwBlock;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(ew_kernel, dim3(static_cast<unsigned>(blocks)), dim3(kEwBlock), 0,
                       reinterpret_cast<hipStream_t>(stream), a);
    return launched(BR_EW_SEG, "flame_elementwise_segments");
}

// the host-side check of a program (both entry points): every register defined before it is read,
// in the dtype the reading op says; every buffer it names present (bufs NULL: the segments'
// buffers are on the device, only the index is checked); an op / dtype the kernel knows
static int ew_check(const flame_ew_op* prog, int32_t n_ops, void* const* bufs, int32_t n_bufs, int64_t numel) {
    if (n_ops < 0 || n_ops > FLAME_EW_MAX_OPS || (n_ops > 0 && !prog))
        return set_err(FLAME_EINVAL, "flame_elementwise: n_ops %d outside [0, %d] or NULL program", n_ops, FLAME_EW_MAX_OPS);
    if (numel < 0) return set_err(FLAME_EINVAL, "flame_elementwise: numel < 0");
    // host-side check of the program: every register defined before it is read, in the dtype the
    // reading op says; every buffer it names present; an op / dtype the kernel knows
    int rdt[FLAME_EW_MAX_REGS];
    for (int k = 0; k < FLAME_EW_MAX_REGS; ++k) rdt[k] = -1;
    auto reg = [](int x) { return x >= 0 && x < FLAME_EW_MAX_REGS; };
    for (int32_t k = 0; k < n_ops; ++k) {
        const flame_ew_op& o = prog[k];
        const int dt = o.dtype;
        if (dt < FLAME_F32 || dt > FLAME_BOOL) return set_err(FLAME_EINVAL, "flame_elementwise: op %d: dtype %d", k, dt);
        auto bad = [&](const char* why) { return set_err(FLAME_EINVAL, "flame_elementwise: op %d (%d): %s", k, o.op, why); };
        switch (o.op) {
        case FLAME_EW_LOAD:
            if (!reg(o.dst) || o.a < 0 || o.a >= n_bufs || (bufs && numel > 0 && !bufs[o.a])) return bad("bad register or buffer");
            rdt[o.dst] = dt;
            break;
        case FLAME_EW_STORE:
            if (!reg(o.b) || o.a < 0 || o.a >= n_bufs || (bufs && numel > 0 && !bufs[o.a])) return bad("bad register or buffer");
            if (rdt[o.b] != dt) return bad("stored register is not of the buffer's dtype");
            break;
        case FLAME_EW_ZERO:
            if (!reg(o.dst)) return bad("bad register");
            rdt[o.dst] = dt;
            break;
        case FLAME_EW_CAST:
            if (!reg(o.dst) || !reg(o.a) || rdt[o.a] < 0 || rdt[o.a] != o.b) return bad("source register undefined or not of dtype b");
            rdt[o.dst] = dt;
            break;
        case FLAME_EW_ADD: case FLAME_EW_SUB: case FLAME_EW_MUL: case FLAME_EW_DIV:
            if (!reg(o.dst) || !reg(o.a) || !reg(o.b) || rdt[o.a] != dt || rdt[o.b] != dt) return bad("operand not of the op's dtype");
            if (o.op == FLAME_EW_DIV && !ew_float(dt)) return bad("division in an integer dtype");
            // bool: torch's + is a logical or, * a logical and (the sum / product != 0); - raises
            if (dt == FLAME_BOOL && o.op == FLAME_EW_SUB) return bad("subtraction in bool");
            rdt[o.dst] = dt;
            break;
        case FLAME_EW_ADD_S: case FLAME_EW_MUL_S: case FLAME_EW_SQUARE: case FLAME_EW_SIGN: case FLAME_EW_SQRT:
            if (!reg(o.dst) || !reg(o.a) || rdt[o.a] != dt) return bad("operand not of the op's dtype");
            if (o.op == FLAME_EW_SQRT && !ew_float(dt)) return bad("sqrt in an integer dtype");
            if (dt == FLAME_BOOL && (o.op == FLAME_EW_ADD_S || o.op == FLAME_EW_MUL_S))
                return bad("a scalar op in bool");
            rdt[o.dst] = dt;
            break;
        default: return bad("unknown op");
        }
    }
    return FLAME_OK;
}

static int check_tile_copies(const flame_tile_copy* t, int32_t n, const char* who) {
    if (n < 0 || (n > 0 && !t)) return set_err(FLAME_EINVAL, "%s: NULL table or n_entries < 0", who);
    for (int32_t i = 0; i < n; ++i) {
        if (t[i].nbytes < 0) return set_err(FLAME_EINVAL, "%s: entry %d: nbytes < 0", who, i);
        if (t[i].nbytes == 0) continue;
        if (!t[i].src || !t[i].dst) return set_err(FLAME_EINVAL, "%s: entry %d: NULL pointer", who, i);
        if (reinterpret_cast<uintptr_t>(t[i].dst) % 16)
            return set_err(FLAME_EINVAL, "%s: entry %d: dst not 16-byte aligned", who, i);
        if (t[i].nbytes > FLAME_TILE_BYTES && (t[i].dst_tile_stride < FLAME_TILE_BYTES || t[i].dst_tile_stride % 16))
            return set_err(FLAME_EINVAL, "%s: entry %d: dst_tile_stride %lld must be >= %d and a multiple of 16", who,
                           i, static_cast<long long>(t[i].dst_tile_stride), FLAME_TILE_BYTES);
    }
    return FLAME_OK;
}

int flame_slab_write(const flame_tile_copy* table, int32_t n_entries, void* stream) {
    int rc = check_tile_copies(table, n_entries, "flame_slab_write");
    if (rc) return rc;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    g_err[0] = 0;
    int32_t i = 0;
    while (i < n_entries) {           // up to kSlabMaxEntries keys per launch (one launch for most models)
        ArgMeta m;
        SlabEntry* ents = reinterpret_cast<SlabEntry*>(m.w);
        int n = 0;
        int64_t tiles = 0;
        for (; i < n_entries && n < kSlabMaxEntries; ++i) {
            if (table[i].nbytes == 0) continue;
            ents[n] = SlabEntry{static_cast<const uint8_t*>(table[i].src), static_cast<uint8_t*>(table[i].dst),
                                table[i].nbytes, table[i].dst_tile_stride, tiles};
            tiles += (table[i].nbytes + FLAME_TILE_BYTES - 1) / FLAME_TILE_BYTES;
            ++n;
        }
        if (n == 0) break;
        const int64_t blocks = (tiles + kSlabTPW - 1) / kSlabTPW;
        if (blocks > 0x7FFFFFFFll) return set_err(FLAME_EINVAL, "flame_slab_write: %lld tiles", (long long)tiles);
        hipLaunchKernelGGL(slab_write_kernel, dim3(static_cast<unsigned>(blocks)), dim3(kBlock), 0, st, m, n, tiles);
        rc = check_launch("flame_slab_write");
        if (rc) return rc;
    }
    return FLAME_OK;
}

int flame_slab_write_2d(const flame_tile_copy* table, int32_t n_entries, void* stream) {
    int rc = check_tile_copies(table, n_entries, "flame_slab_write_2d");
    if (rc) return rc;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    for (int32_t i = 0; i < n_entries; ++i) {
        const flame_tile_copy& t = table[i];
        if (t.nbytes == 0) continue;
        const int64_t full = t.nbytes / FLAME_TILE_BYTES, rem = t.nbytes % FLAME_TILE_BYTES;
        hipError_t e = hipSuccess;
        if (full)
            e = hipMemcpy2DAsync(t.dst, static_cast<size_t>(t.dst_tile_stride), t.src, FLAME_TILE_BYTES,
                                 FLAME_TILE_BYTES, static_cast<size_t>(full), hipMemcpyDefault, st);
        if (e == hipSuccess && rem)
            e = hipMemcpyAsync(static_cast<uint8_t*>(t.dst) + full * t.dst_tile_stride,
                               static_cast<const uint8_t*>(t.src) + full * FLAME_TILE_BYTES, static_cast<size_t>(rem),
                               hipMemcpyDefault, st);
        if (e != hipSuccess) return set_err(FLAME_EHIP, "flame_slab_write_2d: entry %d: %s", i, hipGetErrorString(e));
    }
    g_err[0] = 0;
    return FLAME_OK;
}

int32_t flame_launch_branches(void) { return BR_COUNT; }

const char* flame_launch_branch_name(int32_t branch) { return branch_name(branch); }

int64_t flame_launch_branch_count(int32_t branch) {
    if (branch < 0 || branch >= BR_COUNT) return -1;
    return g_launches[branch].load(std::memory_order_relaxed);
}

}  // extern "C"
