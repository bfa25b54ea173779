// fedagg.hip -- CDNA4 (gfx950) kernels + C ABI for flame's server-side aggregation.
//
// Hot path: the weighted reduction of N client updates into
// one global model, restated from /root/reference/lib/python/flame/
//   optimizer/fedavg.py:79-104, optimizer/fedbuff.py:89-97,122-157,
//   optimizer/fedopt.py:102-129 (+ fedadam.py:33-35, fedyogi.py:34-36, fedadagrad.py:33-35).
//
// Design:
//   * HBM-read bound (≈1 flop per byte): no MFMA, no LDS; every byte is read once.
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
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <cstdarg>
#include <type_traits>

#include "../../include/flame_amd.h"

namespace {

// Tunables (compile-time; defaults chosen by tools/kernel_sweep.py on MI355X)
#ifndef FLAME_BLOCK
#define FLAME_BLOCK 256   // lanes per workgroup of the reduction kernels
#endif
#ifndef FLAME_CU
#define FLAME_CU 8        // clients whose loads are issued together per lane
#endif
#ifndef FLAME_CU16
#define FLAME_CU16 FLAME_CU  // client unroll for 16-bit dtypes (8 elements per lane vector)
#endif
#ifndef FLAME_VPT
#define FLAME_VPT 1       // 16-byte vectors per lane per client (block-strided)
#endif
#ifndef FLAME_PIPE
#define FLAME_PIPE 0      // 1: prefetch the next client batch before combining the current one
#endif
#ifndef FLAME_BF16_HI
#define FLAME_BF16_HI 0   // 1: bf16 rounding as one v_cvt_pk_bf16_f32 into the high half (bf16_round)
#endif
#ifndef FLAME_BF16_PK
#define FLAME_BF16_PK 0   // 1: bf16 client combine on packed fp32 pairs (reduce_clients)
#endif
#ifndef FLAME_DYN_OCC_LDS
#define FLAME_DYN_OCC_LDS 0  // sweep: dynamic LDS bytes per FedDyn workgroup (caps its residency; unused)
#endif
#ifndef FLAME_HLO
#define FLAME_HLO 1       // flame_hier_fedbuff, one middle over >= 64 arrivals and >= 4,096 chunks: low residency
#endif
#ifndef FLAME_HXP
#define FLAME_HXP 0       // hierarchy kernel (LDS store groups, FedBuff mode): > 0 = one double-buffered stream
                          // of that many arrivals per batch across the middles (must divide the arrivals)
#endif
#ifndef FLAME_SPF
#define FLAME_SPF 0       // 1: prefetch the next client batch's pointers (scalar loads) behind the current
                          // batch's vector loads (reduce_clients, vector path)
#endif
#ifndef FLAME_TAILB
#define FLAME_TAILB 0     // 1: the init-first client joins the first batch and the last n % CU clients
                          // load together (reduce_clients, vector path)
#endif
#ifndef FLAME_NT
#define FLAME_NT 1        // non-temporal client loads (read once)
#endif
#ifndef FLAME_ST_NT
#define FLAME_ST_NT 4     // output store policy: 0 plain, 1 nt, 2 sc1, 3 sc0 sc1, 4 sc0 sc1 nt (see st_v)
#endif
#ifndef FLAME_NOSTORE
#define FLAME_NOSTORE 0   // DIAGNOSTIC sweep variant only: skip the reduction's output store
#endif
#ifndef FLAME_WGC
#define FLAME_WGC 1       // chunks per workgroup of the reduction kernel
#endif
#ifndef FLAME_DEFER_ST
#define FLAME_DEFER_ST 0  // 1: store a workgroup's FLAME_WGC output chunks together at its end
#endif
#ifndef FLAME_HCU16
#define FLAME_HCU16 4     // client unroll of the hierarchy kernel for 16-bit dtypes (with FLAME_HBATCH 8:
                          // 90 VGPRs, 5 waves/SIMD; unroll 8 needs 123 VGPRs for the same time)
#endif
#ifndef FLAME_HWPE
#define FLAME_HWPE 0      // hierarchy kernel: minimum waves per SIMD to compile for (0 = compiler's choice)
#endif
#ifndef FLAME_HPF
#define FLAME_HPF 0       // hierarchy kernel: load each middle's weights before its arrival loop
#endif
#ifndef FLAME_HDIAG
#define FLAME_HDIAG 0     // DIAGNOSTIC sweep variants only: 1 = skip middle-weight stores, 2 = also skip their loads
#endif
#ifndef FLAME_BUFLD
#define FLAME_BUFLD 0     // sweep: client loads as buffer loads, cache policy FLAME_BUFLD - 1 (0 = global loads)
#endif
#ifndef FLAME_HTIME
#define FLAME_HTIME 0     // DIAGNOSTIC: per-workgroup timestamps of the hierarchy kernel (wave 0, lane 0;
                          // s_memrealtime, 100 MHz) into the buffer flame_sweep_htime() sets
                          // (tools/hier_attrib.py): start, end, hw ids, each middle's reduction and
                          // epilogue ends, each LDS store burst's end
#endif
#ifndef FLAME_HNX
#define FLAME_HNX 0       // hierarchy kernel (LDS store groups, FedBuff mode): the next middle's first batch of
                          // arrivals is loaded BEFORE the current middle's epilogue (weights load, scale_add,
                          // delta, top), so loads stay in flight across it; whole batches only (the remainder
                          // loads together)
#endif
#ifndef FLAME_HBATCH
#define FLAME_HBATCH 8    // hierarchy kernel: middles whose weight stores are issued together
                          // (C5 shard: 8 -> -1.3..1.6 % vs 1, tools/hier_sweep.py; 16+ spills)
#endif
#ifndef FLAME_HLDS
#define FLAME_HLDS 1      // hierarchy kernel, launches with >= FLAME_HLDS_MIN_MIDS middles: 1 = hold a store
                          // group of FLAME_HLDS_BATCH middles' weights in LDS (4 KiB each per workgroup,
                          // 2 workgroups per CU) instead of FLAME_HBATCH in registers, arrivals unrolled
                          // by FLAME_HLDS_CU16 (C5 shard: 20.99 -> 19.51 ms, 0.7 % above the no-store
                          // diagnostic; tools/hier_sweep.py, profiles/r02_hier_lds_sweep.log)
#endif
#ifndef FLAME_HLDS_BATCH
#define FLAME_HLDS_BATCH 16
#endif
#ifndef FLAME_HLDS_CU16
#define FLAME_HLDS_CU16 6
#endif
#ifndef FLAME_HLDS_MIN_MIDS
#define FLAME_HLDS_MIN_MIDS 16
#endif
#ifndef FLAME_HST
#define FLAME_HST FLAME_ST_NT  // hierarchy kernel: store policy of the middle weights (encoding of FLAME_ST_NT)
#endif
#ifndef FLAME_DYN_CU
#define FLAME_DYN_CU 4    // FedDyn kernel: program steps whose loads are issued together
#endif
#ifndef FLAME_DYN_LDS
#define FLAME_DYN_LDS 0   // FedDyn kernel: > 0 = hold the updated histories of that many program steps in
                          // LDS (4 KiB each per workgroup) and store them in one burst (multiple of FLAME_DYN_CU)
#endif
#ifndef FLAME_DYN_XCD
#define FLAME_DYN_XCD 1   // FedDyn kernel: XCD-contiguous chunk map (see FLAME_AGG_XCD_MAP); histories are
                          // per-end rows by default: 512 x 12M fp32 -0.7 % (cache order) / -1.4 %
                          // (other order), tools/feddyn_sweep.py, profiles/r02_feddyn_xcd_sweep.log
#endif
#ifndef FLAME_DYN_ST
#define FLAME_DYN_ST FLAME_ST_NT  // FedDyn kernel: store policy of the updated histories
#endif
#ifndef FLAME_OCC_LDS
#define FLAME_OCC_LDS 0   // sweep variants: dynamic LDS bytes per reduction / hierarchy workgroup (caps
                          // resident workgroups per CU at 160 KiB / FLAME_OCC_LDS; the kernels use no LDS)
#endif
#ifndef FLAME_LO_CU
#define FLAME_LO_CU 3     // flame_agg_reduce, launches of >= FLAME_LO_MIN_CLIENTS clients and >= FLAME_LO_MIN_CHUNKS
                          // chunks: 2 workgroups per CU (FLAME_LO_LDS of dynamic LDS, unused) with this client
                          // unroll -- fewer loads in flight reads HBM faster (C3: 14.90 -> 14.18 ms, 7.24 TB/s =
                          // 99 % of a region probe at that residency; tools/kernel_sweep.py occ2cu3 / lo0,
                          // profiles/r03ze_c3_sweep.log, r03zf_c3_sweep.log); 0 = off
#endif
#ifndef FLAME_LO_CU16
#define FLAME_LO_CU16 4   // the same for 16-bit dtypes (8 elements per load: unroll 3 reads 6.49 TB/s, 4 6.99;
                          // bf16 1024 x 25M, profiles/r03zf_c3_bf16_sweep.log)
#endif
#ifndef FLAME_LO_LDS
#define FLAME_LO_LDS 65536
#endif
#ifndef FLAME_LO_MIN_CLIENTS
#define FLAME_LO_MIN_CLIENTS 64  // 64 x 100M fp32: 4.04 -> 3.90 ms, bf16 64 x 200M: 4.09 -> 4.00 ms
                                 // (profiles/r03zn_c64_lomin.log, r03zn_b64_lomin.log)
#endif
#ifndef FLAME_LO_MIN_CHUNKS
#define FLAME_LO_MIN_CHUNKS 4096
#endif
#ifndef FLAME_XCD_SWIZZLE
#define FLAME_XCD_SWIZZLE 0  // sweep variant: each XCD (workgroups are dispatched to XCDs round-robin)
                             // streams one contiguous eighth of the chunks
#endif
#ifndef FLAME_OPT_PREFETCH
#define FLAME_OPT_PREFETCH 0  // FedOPT: issue the cur/m/v loads before the client loop
#endif
#ifndef FLAME_OPT_WGC
#define FLAME_OPT_WGC 4   // FedOPT (fp32, >= 8 x 256 x WGC chunks): chunks per workgroup; > 1 holds their
                          // avg/m/v/cur blocks in LDS (16 KiB per chunk; 64 KiB at 4 -> two workgroups
                          // per CU) and stores them in one burst at the end.  C4 FedAdam, tiled slab:
                          // 1 chunk 15.18, 8 chunks (one workgroup per CU, unroll 8) 14.62 ms (round 2,
                          // profiles/r02_fedopt_wgc_sweep.log); 4 chunks with unroll 3 (fewer loads in
                          // flight, as flame_agg_reduce's FLAME_LO_CU) 1.8-2.0 % under 8 chunks / unroll 8
                          // (profiles/r03zf_c4_sweep.log, r03zg_c4_sweep.log)
#endif
#ifndef FLAME_OPT_CU
#define FLAME_OPT_CU 3    // FedOPT fp32 client unroll with FLAME_OPT_WGC > 1
#endif

constexpr int kBlock = FLAME_BLOCK;
#if FLAME_HTIME
__device__ uint64_t* g_htime = nullptr;
__device__ int g_htime_slots = 0;
__device__ __forceinline__ void htime(int slot, uint64_t v) {
    if (threadIdx.x == 0 && g_htime && slot < g_htime_slots)
        g_htime[static_cast<int64_t>(blockIdx.x) * g_htime_slots + slot] = v;
}
#define FLAME_HT(slot) htime((slot), __builtin_amdgcn_s_memrealtime())
#else
#define FLAME_HT(slot) do {} while (0)
#endif
constexpr int kHB = FLAME_HBATCH;
constexpr int kVPT = FLAME_VPT;
constexpr int kWGC = FLAME_WGC;
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
#if FLAME_BF16_HI
    // RNE fp32 -> bf16 -> fp32 in ONE instruction: v_cvt_pk_bf16_f32 packs (lo, hi) = (bf16(0),
    // bf16(x)), and that dword IS the fp32 value of bf16(x) (the compiler's lowering of the cast
    // puts x in the low half and shifts it back up: two instructions per rounding)
    float r;
    asm("v_cvt_pk_bf16_f32 %0, 0, %1" : "=v"(r) : "v"(x));
    return r;
#else
    // RNE fp32 -> bf16 -> fp32 (v_cvt_pk_bf16_f32 on gfx950)
    return static_cast<float>(static_cast<__bf16>(x));
#endif
}
__device__ __forceinline__ float bf16_to_f32(uint16_t b) {
    return __uint_as_float(static_cast<uint32_t>(b) << 16);
}
__device__ __forceinline__ uint16_t f32_to_bf16_exact(float x) {  // x already bf16-representable
    return static_cast<uint16_t>(__float_as_uint(x) >> 16);
}
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

__device__ __forceinline__ V16 ld_nt(const void* p) {
#if FLAME_NT
    u4 x = __builtin_nontemporal_load(G(reinterpret_cast<const u4*>(p)));
#else
    u4 x = *G(reinterpret_cast<const u4*>(p));
#endif
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
#if FLAME_ST_NT == 1
    __builtin_nontemporal_store(x, G(reinterpret_cast<u4*>(p)));
#elif FLAME_ST_NT == 2
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" :: "v"(p), "v"(x) : "memory");
#elif FLAME_ST_NT == 3
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" :: "v"(p), "v"(x) : "memory");
#elif FLAME_ST_NT == 4
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt\n\ts_nop 1" :: "v"(p), "v"(x) : "memory");
#else
    *G(reinterpret_cast<u4*>(p)) = x;
#endif
}
// Store with an explicit policy (same encoding as FLAME_ST_NT).
template <int POL>
__device__ __forceinline__ void st_pol(void* p, const V16& v) {
    u4 x = {v.w[0], v.w[1], v.w[2], v.w[3]};
    if constexpr (POL == 1) {
        __builtin_nontemporal_store(x, G(reinterpret_cast<u4*>(p)));
    } else if constexpr (POL == 2) {
        asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" :: "v"(p), "v"(x) : "memory");
    } else if constexpr (POL == 3) {
        asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" :: "v"(p), "v"(x) : "memory");
    } else if constexpr (POL == 4) {
        asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt\n\ts_nop 1" :: "v"(p), "v"(x) : "memory");
    } else if constexpr (POL == 5) {
        asm volatile("global_store_dwordx4 %0, %1, off nt sc1\n\ts_nop 1" :: "v"(p), "v"(x) : "memory");
    } else {
        *G(reinterpret_cast<u4*>(p)) = x;
    }
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
#if FLAME_BUFLD
        if constexpr (VEC) {
            // buffer loads: the client's chunk base (wave-uniform) in a scalar resource, the
            // lane's byte offset in one VGPR; FLAME_BUFLD - 1 = cache policy (sc0 1, nt 2, sc1 16)
            const int32_t lane_b = static_cast<int32_t>(threadIdx.x) * EPT * static_cast<int32_t>(sizeof(T));
            const uint64_t wb = cp[c] + static_cast<uint64_t>(coff - lane_b);
            const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(wb));
            const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(wb >> 32));
            void* base = reinterpret_cast<void*>((static_cast<uint64_t>(hi) << 32) | lo);
            __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, 0x7fffffff, 0x00020000);
#pragma unroll
            for (int v = 0; v < kVPT; ++v) {
                u4 q = __builtin_amdgcn_raw_buffer_load_b128(r, lane_b + v * static_cast<int32_t>(VS * sizeof(T)), 0,
                                                             FLAME_BUFLD - 1);
                V16 t;
                t.w[0] = q[0]; t.w[1] = q[1]; t.w[2] = q[2]; t.w[3] = q[3];
                unpack<T, EPT>(t, x[v]);
            }
            return;
        }
#endif
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
#if FLAME_BF16_PK
        if constexpr (DT == FLAME_BF16) {
            // the same two roundings per element, two elements per packed-fp32 multiply and add
            // (v_pk_mul_f32 / v_pk_add_f32: each lane's result is the IEEE fp32 op's)
            using f2 = __attribute__((ext_vector_type(2))) float;
            const f2 r2 = {r, r};
#pragma unroll
            for (int v = 0; v < kVPT; ++v)
#pragma unroll
                for (int j = 0; j < EPT; j += 2) {
                    const f2 x2 = {X::ld(x[v][j]), X::ld(x[v][j + 1])};
                    f2 t2 = x2 * r2;
                    t2 = f2{bf16_round(t2.x), bf16_round(t2.y)};
                    f2 a2 = f2{acc[v][j], acc[v][j + 1]} + t2;
                    acc[v][j] = bf16_round(a2.x);
                    acc[v][j + 1] = bf16_round(a2.y);
                }
            return;
        }
#endif
#pragma unroll
        for (int v = 0; v < kVPT; ++v)
#pragma unroll
            for (int j = 0; j < EPT; ++j) acc[v][j] = X::add(acc[v][j], X::tmp(x[v][j], r, rd));
    };
    auto combine = [&](int c, const T (&x)[kVPT][EPT]) { combine_r(rate32(c), rate64(c), x); };
#if FLAME_SPF
    if constexpr (VEC && CU > 1 && DT != FLAME_F64) {
        // the next batch's client pointers AND rates are read (scalar loads) while the current
        // batch's vector loads are in flight: a batch never waits on its pointer row before
        // issuing, nor its combine on a rate load (a rate loaded in the combine, as the plain
        // loop does, makes the combine's lgkmcnt(0) wait for every scalar load in flight, the
        // prefetched pointers included).  Scalar-cache misses matter once a launch's pointer
        // and rate rows outgrow the scalar cache (4,096 arrivals: 48 KiB per workgroup)
        if (init_first && n > 0) {    // the init-first client's load goes out with the first batch
            const int r = n < CU ? n : CU;
            T x[CU][kVPT][EPT];
#pragma unroll
            for (int u = 0; u < CU; ++u)
                if (u < r) load_client(u, x[u]);
            const float r0 = rate32(0);
#pragma unroll
            for (int v = 0; v < kVPT; ++v)
#pragma unroll
                for (int j = 0; j < EPT; ++j) acc[v][j] = X::tmp(x[0][v][j], r0, 0.0);
#pragma unroll
            for (int u = 1; u < CU; ++u)
                if (u < r) combine(u, x[u]);
            i = r;
        }
        if (i + CU <= n) {
            uint64_t pa[CU];
            float ra[CU];
#pragma unroll
            for (int u = 0; u < CU; ++u) {
                pa[u] = cp[i + u];
                ra[u] = r32[i + u];
            }
            while (true) {
                T x[CU][kVPT][EPT];
#pragma unroll
                for (int u = 0; u < CU; ++u) {
                    const T* p = reinterpret_cast<const T*>(reinterpret_cast<const char*>(pa[u]) + coff);
#pragma unroll
                    for (int v = 0; v < kVPT; ++v) unpack<T, EPT>(ld_nt(p + v * VS), x[u][v]);
                }
                float rc[CU];
#pragma unroll
                for (int u = 0; u < CU; ++u) rc[u] = ra[u];
                const bool more = i + 2 * CU <= n;
                if (more) {
#pragma unroll
                    for (int u = 0; u < CU; ++u) {
                        pa[u] = cp[i + CU + u];
                        ra[u] = r32[i + CU + u];
                    }
                }
#pragma unroll
                for (int u = 0; u < CU; ++u) combine_r(rc[u], 0.0, x[u]);
                i += CU;
                if (!more) break;
            }
        }
        if (i < n) {                  // the last n % CU clients' loads go out together
            const int r = n - i;
            T x[CU][kVPT][EPT];
#pragma unroll
            for (int u = 0; u < CU; ++u)
                if (u < r) load_client(i + u, x[u]);
#pragma unroll
            for (int u = 0; u < CU; ++u)
                if (u < r) combine(i + u, x[u]);
        }
        return;
    }
#endif
#if FLAME_TAILB
    if constexpr (VEC && CU > 1) {
        // whole batches only: the init-first client's load goes out with the first batch and the
        // last n % CU clients' loads go out together (one wait each, not one round trip per
        // client); the arithmetic is the same sequence, in client order
        if (init_first && n > 0) {
            const int r = n < CU ? n : CU;
            T x[CU][kVPT][EPT];
#pragma unroll
            for (int u = 0; u < CU; ++u)
                if (u < r) load_client(u, x[u]);
            const float r0 = rate32(0);
            const double rd0 = rate64(0);
#pragma unroll
            for (int v = 0; v < kVPT; ++v)
#pragma unroll
                for (int j = 0; j < EPT; ++j) acc[v][j] = X::tmp(x[0][v][j], r0, rd0);
#pragma unroll
            for (int u = 1; u < CU; ++u)
                if (u < r) combine(u, x[u]);
            i = r;
        }
        for (; i + CU <= n; i += CU) {
            T x[CU][kVPT][EPT];
#pragma unroll
            for (int u = 0; u < CU; ++u) load_client(i + u, x[u]);
#pragma unroll
            for (int u = 0; u < CU; ++u) combine(i + u, x[u]);
        }
        if (i < n) {
            const int r = n - i;
            T x[CU][kVPT][EPT];
#pragma unroll
            for (int u = 0; u < CU; ++u)
                if (u < r) load_client(i + u, x[u]);
#pragma unroll
            for (int u = 0; u < CU; ++u)
                if (u < r) combine(i + u, x[u]);
        }
        return;
    }
#endif
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
#if FLAME_PIPE
    if (VEC && i + CU <= n) {
        // two register batches: batch k+1's loads are in flight while batch k is combined
        T xa[CU][kVPT][EPT], xb[CU][kVPT][EPT];
#pragma unroll
        for (int u = 0; u < CU; ++u) load_client(i + u, xa[u]);
        while (true) {
            const bool nb = i + 2 * CU <= n;
            if (nb) {
#pragma unroll
                for (int u = 0; u < CU; ++u) load_client(i + CU + u, xb[u]);
            }
#pragma unroll
            for (int u = 0; u < CU; ++u) combine(i + u, xa[u]);
            i += CU;
            if (!nb) break;
            const bool na = i + 2 * CU <= n;
            if (na) {
#pragma unroll
                for (int u = 0; u < CU; ++u) load_client(i + CU + u, xa[u]);
            }
#pragma unroll
            for (int u = 0; u < CU; ++u) combine(i + u, xb[u]);
            i += CU;
            if (!na) break;
        }
    }
#endif
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
    for (int v = 0; v < kVPT; ++v) {
#if FLAME_NOSTORE
        if (__builtin_expect(ov[v].w[0] == 0x12345u && ov[v].w[1] == 0x54321u, 0))   // keeps the math live
#endif
        st_v(op + v * VS, ov[v]);
    }
}

// Workgroup slot of block b when the 8 XCDs (dispatched round-robin) each take one
// contiguous eighth of the slots (FLAME_AGG_XCD_MAP / FLAME_OPT_XCD_MAP): a bijection.
__device__ __forceinline__ int64_t xcd_slot(int64_t b, int64_t n) {
    const int64_t q = n / 8, r = n % 8, x = b % 8;
    return x * q + (x < r ? x : r) + b / 8;
}

// Workgroup w reduces chunks [w*kWGC, (w+1)*kWGC).  With FLAME_DEFER_ST the full
// chunks' output vectors stay in registers and are stored together at the end.
template <int DT, int CU>
__device__ __forceinline__ void agg_reduce_body(const flame_segment* __restrict__ segs, int n_segs,
                                                const uint64_t* __restrict__ clients, int n_clients,
                                                const float* __restrict__ r32, const double* __restrict__ r64,
                                                unsigned flags, int64_t n_chunks) {
    using T = typename Tr<DT>::T;
#if FLAME_DEFER_ST
    V16 ov[kWGC][kVPT];
    T* op[kWGC];
    bool full[kWGC];
#pragma unroll
    for (int k = 0; k < kWGC; ++k) {
        const int64_t chunk = static_cast<int64_t>(blockIdx.x) * kWGC + k;
        full[k] = chunk < n_chunks &&
                  reduce_chunk<DT, CU>(segs, n_segs, clients, n_clients, r32, r64, flags, chunk, ov[k], op[k]);
    }
#pragma unroll
    for (int k = 0; k < kWGC; ++k)
        if (full[k]) store_chunk(op[k], ov[k]);
#else
    const int64_t wg = (FLAME_XCD_SWIZZLE || (flags & FLAME_AGG_XCD_MAP)) ? xcd_slot(blockIdx.x, gridDim.x)
                                                                           : blockIdx.x;
#pragma unroll 1
    for (int k = 0; k < kWGC; ++k) {
        const int64_t chunk = wg * kWGC + k;
        if (chunk >= n_chunks) break;
        V16 ov[kVPT];
        T* op;
        if (reduce_chunk<DT, CU>(segs, n_segs, clients, n_clients, r32, r64, flags, chunk, ov, op))
            store_chunk(op, ov);
    }
#endif
}

template <int DT, int CU>
__global__ __launch_bounds__(kBlock) void agg_reduce_kernel(const flame_segment* __restrict__ segs, int n_segs,
                                                            const uint64_t* __restrict__ clients, int n_clients,
                                                            const float* __restrict__ r32,
                                                            const double* __restrict__ r64, unsigned flags,
                                                            int64_t n_chunks) {
    agg_reduce_body<DT, CU>(segs, n_segs, clients, n_clients, r32, r64, flags, n_chunks);
}

// Small launches (few segments x few hundred clients): the whole metadata block travels as a
// kernel argument.  A separate H2D copy of a few KB is a blit kernel on gfx950 that the launch
// stream must run before the reduction (≈15 µs of GPU timeline per launch, measured on
// config 2: 0.171 -> 0.157 ms per step without it); kernel arguments reach the GPU with the
// dispatch itself and are read through the scalar cache like the device-resident table.
constexpr int kArgMetaWords = 448;          // 3,584 B: kernel arguments are limited to 4 KiB
struct ArgMeta { uint64_t w[kArgMetaWords]; };

template <int DT, int CU>
__global__ __launch_bounds__(kBlock) void agg_reduce_kernel_argmeta(const ArgMeta meta, int n_segs, int n_clients,
                                                                    int off_clients, int off_r32, int off_r64,
                                                                    unsigned flags, int64_t n_chunks) {
    // `meta` is the first kernel argument: read it in place in the kernarg segment (scalar
    // loads) -- naming the by-value parameter would copy 3.5 KB into every lane's scratch
    (void)sizeof(meta);
    const uint64_t* w = (const uint64_t*)__builtin_amdgcn_kernarg_segment_ptr();
    agg_reduce_body<DT, CU>(reinterpret_cast<const flame_segment*>(w), n_segs, w + off_clients, n_clients,
                            off_r32 >= 0 ? reinterpret_cast<const float*>(w + off_r32) : nullptr,
                            off_r64 >= 0 ? reinterpret_cast<const double*>(w + off_r64) : nullptr, flags, n_chunks);
}

// ---------------------------------------------------------------- fused FedOPT (fp32)
__device__ __forceinline__ float sign_f(float x) {  // torch.sign: NaN -> 0, -0 -> 0
    return static_cast<float>((0.0f < x) - (x < 0.0f));
}

// Per-dtype rounding after each reference op (identity for fp32; RNE to bf16 / fp16).
template <int DT> __device__ __forceinline__ float rnd(float x) {
    if constexpr (DT == FLAME_BF16) return bf16_round(x);
    else if constexpr (DT == FLAME_F16) return f16_round(x);
    else return x;
}

// One element of fedopt.py:106-129 (+ the _delta_v variants), each torch op rounded in the
// tensor's dtype.  `tau` arrives pre-rounded to the dtype for bf16/fp16 (torch-CPU rounds a
// Python scalar to a reduced-precision tensor's dtype before + and -, not before * and /).
template <int DT, int VARIANT>
__device__ __forceinline__ void adapt_elem(float avg, float cur, float& m, float& v, float& cur_out,
                                           float b1, float omb1, float b2, float omb2, float eta, float tau) {
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
    // __builtin_sqrtf is correctly rounded; the __fsqrt_rn builtin lowers to the 1-ulp v_sqrt_f32
    const float den = rnd<DT>(__fadd_rn(rnd<DT>(__builtin_sqrtf(vn)), tau));
    const float q = rnd<DT>(__fdiv_rn(rnd<DT>(__fmul_rn(eta, mn)), den));
    m = mn;
    v = vn;
    cur_out = rnd<DT>(__fadd_rn(cur, q));
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
#if FLAME_OPT_PREFETCH
        T curs[kVPT][EPT], ms[kVPT][EPT], vs[kVPT][EPT];
#pragma unroll
        for (int v = 0; v < kVPT; ++v) {
            unpack<T, EPT>(ld_v(curp + v * VS), curs[v]);
            if (!zero_state) {
                unpack<T, EPT>(ld_v(mp + v * VS), ms[v]);
                unpack<T, EPT>(ld_v(vp + v * VS), vs[v]);
            }
        }
#endif
        reduce_clients<DT, CU, true>(acc, false, cp, n_clients, r32, nullptr, e0, sg.numel, coff);
#pragma unroll
        for (int v = 0; v < kVPT; ++v) {
            T cur_t[EPT], m_t[EPT], v_t[EPT], avg_o[EPT], m_o[EPT], v_o[EPT], c_o[EPT];
#if FLAME_OPT_PREFETCH
#pragma unroll
            for (int j = 0; j < EPT; ++j) { cur_t[j] = curs[v][j]; m_t[j] = ms[v][j]; v_t[j] = vs[v][j]; }
#else
            unpack<T, EPT>(ld_v(curp + v * VS), cur_t);
            if (!zero_state) {
                unpack<T, EPT>(ld_v(mp + v * VS), m_t);
                unpack<T, EPT>(ld_v(vp + v * VS), v_t);
            }
#endif
#pragma unroll
            for (int j = 0; j < EPT; ++j) {
                float mj = zero_state ? 0.f : X::ld(m_t[j]), vj = zero_state ? 0.f : X::ld(v_t[j]), cj;
                adapt_elem<DT, VARIANT>(acc[v][j], X::ld(cur_t[j]), mj, vj, cj, b1, omb1, b2, omb2, eta, tau);
                avg_o[j] = X::st(acc[v][j]);
                m_o[j] = X::st(mj);
                v_o[j] = X::st(vj);
                c_o[j] = X::st(cj);
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
                adapt_elem<DT, VARIANT>(acc[v][j], X::ld(ld1(curp + o)), mj, vj, cj, b1, omb1, b2, omb2, eta, tau);
                if (ap) st1(ap + o, X::st(acc[v][j]));
                st1(mp + o, X::st(mj));
                st1(vp + o, X::st(vj));
                st1(cop + o, X::st(cj));
            }
    }
    return false;
}

// G = 1: one chunk per workgroup, stored as computed.  G > 1: G consecutive chunks per
// workgroup, their outputs held in LDS and stored together at the end (FLAME_OPT_WGC).
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
        static_assert(G * 4 * kVPT * kBlock * sizeof(V16) <= 160 * 1024, "FLAME_OPT_WGC: outputs exceed the LDS");
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
template <int DT, int VARIANT, int CU>
__global__ __launch_bounds__(kBlock) void fedopt_kernel_argmeta(const ArgMeta meta, int n_segs, int n_clients,
                                                                int off_clients, int off_r32, unsigned flags,
                                                                float b1, float omb1, float b2, float omb2,
                                                                float eta, float tau) {
    (void)sizeof(meta);
    const uint64_t* w = (const uint64_t*)__builtin_amdgcn_kernarg_segment_ptr();
    fedopt_body<DT, VARIANT, CU, 1>(reinterpret_cast<const flame_segment*>(w), n_segs, w + off_clients, n_clients,
                                    off_r32 >= 0 ? reinterpret_cast<const float*>(w + off_r32) : nullptr, flags,
                                    b1, omb1, b2, omb2, eta, tau, 0);
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
#if FLAME_HWPE
#define FLAME_HIER_ATTR __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(FLAME_HWPE, 8)))
#else
#define FLAME_HIER_ATTR __launch_bounds__(kBlock)
#endif
// SYNC (FLAME_HIER_SYNC): the synchronous hierarchy instead (syncfl/middle_aggregator.py:163-229,
// syncfl/top_aggregator.py:122-176): each middle's FedAvg starts from its weights,
//   a = w_m + tmp(c_{m,0}, r_{m,0}) + ...;  w_m' = a;  d_m = w_m' - w_m
// and the top's FedAvg adds tmp(d_m, top_rates[m]) to the top weights (top_agg_in).
template <int DT> __device__ __forceinline__ float rnd(float x);
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
        FLAME_HT(0);
#if FLAME_HTIME
        // HW_ID (wave / SIMD / CU / SH / SE) and the XCC id of this workgroup's wave 0
        htime(2, static_cast<uint64_t>(__builtin_amdgcn_s_getreg((31 << 11) | 4)) |
                     (static_cast<uint64_t>(__builtin_amdgcn_s_getreg((15 << 11) | 20)) << 32));
#endif
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
#if FLAME_HXP
        // ONE double-buffered stream of arrival batches across the middles (FLAME_HXP arrivals per
        // batch, dividing n_clients): the next batch -- the next middle's first one included -- is in
        // flight while the current batch is combined and while a finished middle's epilogue runs, so
        // a wave's loads never drain at a middle boundary.  A middle's weights are loaded one middle
        // ahead (with the previous middle's first batch): loads complete in issue order, so a
        // weights load issued behind the current batches would hold the epilogue until they land.
        // Same per-element operation order as the loop below (bitwise).
        constexpr int XB = FLAME_HXP;
        if (HL && !SYNC && kVPT == 1 && n_clients % XB == 0 && n_clients >= XB) {
            const int bpm = n_clients / XB;
            const int nbt = n_mids * bpm;
            T xa[XB][kVPT][EPT], xb[XB][kVPT][EPT];
            V16 wc, wn;
            wc = ld_v(mid_ptr(0));
            if (n_mids > 1) wn = ld_v(mid_ptr(1));
            A acc[kVPT][EPT];
            auto issue = [&](int b, T (&x)[XB][kVPT][EPT]) {
                const int m = b / bpm;
                const int c0 = (b - m * bpm) * XB;
                const uint64_t* cp = crow + static_cast<int64_t>(m) * n_clients + c0;
#pragma unroll
                for (int u = 0; u < XB; ++u) {
                    const T* p = reinterpret_cast<const T*>(reinterpret_cast<const char*>(cp[u]) + coff);
#pragma unroll
                    for (int v = 0; v < kVPT; ++v) unpack<T, EPT>(ld_nt(p + v * VS), x[u][v]);
                }
            };
            auto combine_batch = [&](int b, const T (&x)[XB][kVPT][EPT]) {
                const int m = b / bpm;
                const int c0 = (b - m * bpm) * XB;
                const float* r = mid_rates + static_cast<int64_t>(m) * n_clients + c0;
#pragma unroll
                for (int u = 0; u < XB; ++u) {
                    const float ru = r[u];
#pragma unroll
                    for (int v = 0; v < kVPT; ++v)
#pragma unroll
                        for (int j = 0; j < EPT; ++j) {
                            const A t = X::tmp(x[u][v][j], ru, 0.0);
                            acc[v][j] = (u == 0 && c0 == 0) ? t : X::add(acc[v][j], t);   // init-first
                        }
                }
                if (c0 + XB < n_clients) return;
                // middle m complete: scale_add from its weights, the delta into the top, the new
                // weights into the LDS-held store group (stored as a burst when the group is full)
                T* dp = (drow && drow[m]) ? reinterpret_cast<T*>(drow[m]) + e0 : nullptr;
                const float g = mid_goal[m], rt = top_rates[m];
                const int u = m % HB;
                T w[EPT], d[EPT];
                unpack<T, EPT>(wc, w);
#pragma unroll
                for (int j = 0; j < EPT; ++j) {
                    S::op(w[j], X::st(acc[0][j]), g, static_cast<double>(g), &d[j]);
                    const A t = X::tmp(d[j], rt, 0.0);
                    top[0][j] = have_top ? X::add(top[0][j], t) : t;
                }
                have_top = true;
                held[u * kBlock + threadIdx.x] = pack<T, EPT>(w);
                if (dp) st_v(dp, pack<T, EPT>(d));
                wc = wn;                           // loaded a whole middle ago
                if (m + 2 < n_mids) wn = ld_v(mid_ptr(m + 2));
                if ((u == HB - 1 || m == n_mids - 1) && !(flags & FLAME_HIER_MID_READONLY)) {
                    const int mg = m - u;
#pragma unroll 1
                    for (int q = 0; q <= u; ++q) st_pol<FLAME_HST>(mid_ptr(mg + q), held[q * kBlock + threadIdx.x]);
                }
            };
            issue(0, xa);
            int b = 0;
#pragma unroll 1
            while (true) {
                if (b + 1 < nbt) issue(b + 1, xb);
                combine_batch(b, xa);
                if (++b >= nbt) break;
                if (b + 1 < nbt) issue(b + 1, xa);
                combine_batch(b, xb);
                if (++b >= nbt) break;
            }
        } else
#endif
#if FLAME_HNX
        if (HL && !SYNC && kVPT == 1 && n_clients >= CU) {
            T xf[CU][EPT];        // the next middle's first CU arrivals, loaded ahead
            auto issue_first = [&](int m) {
                const uint64_t* cp = crow + static_cast<int64_t>(m) * n_clients;
#pragma unroll
                for (int u = 0; u < CU; ++u)
                    unpack<T, EPT>(ld_nt(reinterpret_cast<const char*>(cp[u]) + coff), xf[u]);
            };
            issue_first(0);
#pragma unroll 1
            for (int m0 = 0; m0 < n_mids; m0 += HB) {
                const int nb = n_mids - m0 < HB ? n_mids - m0 : HB;
#pragma unroll 1
                for (int u = 0; u < nb; ++u) {
                    const int m = m0 + u;
                    const uint64_t* cp = crow + static_cast<int64_t>(m) * n_clients;
                    const float* rr = mid_rates + static_cast<int64_t>(m) * n_clients;
                    A acc[EPT];
                    {   // init-first: acc = tmp(a_0), then + tmp(a_u) in arrival order
                        const float r0 = rr[0];
#pragma unroll
                        for (int j = 0; j < EPT; ++j) acc[j] = X::tmp(xf[0][j], r0, 0.0);
#pragma unroll
                        for (int q = 1; q < CU; ++q) {
                            const float r = rr[q];
#pragma unroll
                            for (int j = 0; j < EPT; ++j) acc[j] = X::add(acc[j], X::tmp(xf[q][j], r, 0.0));
                        }
                    }
                    int i = CU;
#pragma unroll 1
                    for (; i + CU <= n_clients; i += CU) {
                        T x[CU][EPT];
#pragma unroll
                        for (int q = 0; q < CU; ++q)
                            unpack<T, EPT>(ld_nt(reinterpret_cast<const char*>(cp[i + q]) + coff), x[q]);
#pragma unroll
                        for (int q = 0; q < CU; ++q) {
                            const float r = rr[i + q];
#pragma unroll
                            for (int j = 0; j < EPT; ++j) acc[j] = X::add(acc[j], X::tmp(x[q][j], r, 0.0));
                        }
                    }
                    if (i < n_clients) {      // the remainder's loads go out together
                        const int rem = n_clients - i;
                        T x[CU][EPT];
#pragma unroll
                        for (int q = 0; q < CU; ++q)
                            if (q < rem) unpack<T, EPT>(ld_nt(reinterpret_cast<const char*>(cp[i + q]) + coff), x[q]);
#pragma unroll
                        for (int q = 0; q < CU; ++q) {
                            if (q >= rem) break;
                            const float r = rr[i + q];
#pragma unroll
                            for (int j = 0; j < EPT; ++j) acc[j] = X::add(acc[j], X::tmp(x[q][j], r, 0.0));
                        }
                    }
                    FLAME_HT(3 + 2 * m);
                    // the middle's weights, then the next middle's first batch: both in flight
                    // while this middle's epilogue waits for the weights
                    const V16 wv = ld_v(mid_ptr(m));
                    if (m + 1 < n_mids) issue_first(m + 1);
                    T* dp = (drow && drow[m]) ? reinterpret_cast<T*>(drow[m]) + e0 : nullptr;
                    const float g = mid_goal[m], rt = top_rates[m];
                    T w[EPT], d[EPT];
                    unpack<T, EPT>(wv, w);
#pragma unroll
                    for (int j = 0; j < EPT; ++j) {
                        S::op(w[j], X::st(acc[j]), g, static_cast<double>(g), &d[j]);
                        const A t = X::tmp(d[j], rt, 0.0);
                        top[0][j] = have_top ? X::add(top[0][j], t) : t;
                    }
                    held[u * kBlock + threadIdx.x] = pack<T, EPT>(w);
                    if (dp) st_v(dp, pack<T, EPT>(d));
                    have_top = true;
                    FLAME_HT(4 + 2 * m);
                }
                if (!(flags & FLAME_HIER_MID_READONLY)) {
#pragma unroll 1
                    for (int u = 0; u < nb; ++u) st_pol<FLAME_HST>(mid_ptr(m0 + u), held[u * kBlock + threadIdx.x]);
                }
                FLAME_HT(3 + 2 * n_mids + m0 / HB);
            }
        } else
#endif
#pragma unroll 1
        for (int m0 = 0; m0 < n_mids; m0 += HB) {
            V16 pend[HL ? 1 : HB][kVPT];
            const int nb = n_mids - m0 < HB ? n_mids - m0 : HB;   // middles in this group
#pragma unroll
            for (int u = 0; u < HB; ++u) {
            const int m = m0 + u;
            if (HB > 1 && m >= n_mids) break;
            T* wp = mid_ptr(m);
#if FLAME_HPF
            V16 wv[kVPT];
#pragma unroll
            for (int v = 0; v < kVPT; ++v) wv[v] = ld_v(wp + v * VS);
#endif
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
            FLAME_HT(3 + 2 * m);
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
#if FLAME_HPF
                    unpack<T, EPT>(wv[v], w);
#elif FLAME_HDIAG == 2
#pragma unroll
                    for (int j = 0; j < EPT; ++j) w[j] = T(0);
#else
                    unpack<T, EPT>(ld_v(wp + v * VS), w);
#endif
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
            FLAME_HT(4 + 2 * m);
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
#if FLAME_HDIAG
                        if (__builtin_expect(pv.w[0] == 0x12345u && pv.w[1] == 0x54321u, 0))
#endif
                        st_pol<FLAME_HST>(wp + v * VS, pv);
                    }
                }
            }
            FLAME_HT(3 + 2 * n_mids + m0 / HB);
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
        FLAME_HT(1);
        return;
    }
    // tails / misaligned views: element-wise, same op sequence
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

template <int DT, int CU, bool SYNC, int HB, bool HL>
__global__ FLAME_HIER_ATTR void hier_fedbuff_kernel(const flame_hier_segment* __restrict__ segs, int n_segs,
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
template <int DT, int CU, bool SYNC>
__global__ FLAME_HIER_ATTR void hier_fedbuff_kernel_argmeta(const ArgMeta meta, int n_segs, int n_mids, int n_clients,
                                                            int o_mid_w, int o_mid_delta, int o_clients,
                                                            int o_mid_rates, int o_mid_goal, int o_top_rates,
                                                            float top_goal, unsigned flags) {
    (void)sizeof(meta);     // read in place in the kernarg segment (see agg_reduce_kernel_argmeta)
    const uint64_t* w = (const uint64_t*)__builtin_amdgcn_kernarg_segment_ptr();
    hier_fedbuff_body<DT, CU, SYNC, kHB, false>(reinterpret_cast<const flame_hier_segment*>(w), n_segs, n_mids, n_clients,
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
template <int DT, int CU, bool VEC, int G>
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
    auto store = [&](void* base, int64_t off, const T (&x)[kVPT][EPT], auto pol) {
        constexpr int POL = decltype(pol)::value;
        T* p = reinterpret_cast<T*>(reinterpret_cast<char*>(base) + off);
#pragma unroll
        for (int v = 0; v < kVPT; ++v) {
            if constexpr (VEC) {
                st_pol<POL>(p + v * VS, pack<T, EPT>(x[v]));
            } else {
#pragma unroll
                for (int j = 0; j < EPT; ++j)
                    if (e0 + v * VS + j < sg.numel) st1(p + v * VS + j, x[v][j]);
            }
        }
    };
    using out_pol = std::integral_constant<int, FLAME_ST_NT>;
    using hist_pol = std::integral_constant<int, FLAME_DYN_ST>;
    // G > 0: updated histories wait in LDS (lane-private slots) and go out G steps at a time
    constexpr bool HL = VEC && G > 0;
    static_assert(!HL || G % CU == 0, "FLAME_DYN_LDS must be a multiple of FLAME_DYN_CU");
    __shared__ V16 held[HL ? G * kVPT * kBlock : 1];
    auto flush = [&](int q0, int q1) {
#pragma unroll 1
        for (int q = q0; q < q1; ++q) {
            if (!(sflags[q] & FLAME_DYN_HOUT)) continue;
            T* p = reinterpret_cast<T*>(reinterpret_cast<char*>(row[static_cast<int64_t>(q) * 3 + 2]) + hoff);
#pragma unroll
            for (int v = 0; v < kVPT; ++v) st_pol<FLAME_DYN_ST>(p + v * VS, held[((q - q0) * kVPT + v) * kBlock + threadIdx.x]);
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
        int kg = phase ? n_phase1 : 0;       // first step whose history is still held (HL)
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
                    if constexpr (HL) {
#pragma unroll
                        for (int v = 0; v < kVPT; ++v)
                            held[((k + u - kg) * kVPT + v) * kBlock + threadIdx.x] = pack<T, EPT>(h[u][v]);
                    } else {
                        store(reinterpret_cast<void*>(row[static_cast<int64_t>(k + u) * 3 + 2]), hoff, h[u], hist_pol{});
                    }
                }
                if (f & FLAME_DYN_MEAN) {
#pragma unroll
                    for (int v = 0; v < kVPT; ++v)
#pragma unroll
                        for (int j = 0; j < EPT; ++j) mean[v][j] = X::add(mean[v][j], X::tmp(h[u][v][j], rm32, rm64));
                }
            }
            if constexpr (HL) {     // a full group, or the phase's last steps: store the held histories
                const int k1 = k + nb;
                if (k1 - kg >= G || k1 >= end) {
                    flush(kg, k1);
                    kg = k1;
                }
            }
        }
    }
    T o[kVPT][EPT], c[kVPT][EPT];
#pragma unroll
    for (int v = 0; v < kVPT; ++v)
#pragma unroll
        for (int j = 0; j < EPT; ++j) { o[v][j] = X::st(avg[v][j]); c[v][j] = X::st(X::add(avg[v][j], mean[v][j])); }
    store(sg.out, ooff, o, out_pol{});
    store(sg.cld, ooff, c, out_pol{});
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
    const int64_t chunk = FLAME_DYN_XCD ? xcd_slot(blockIdx.x, gridDim.x) : blockIdx.x;
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
        feddyn_chunk<DT, CU, true, FLAME_DYN_LDS>(sg, row, sflags, n_steps, n_phase1, ra32, rm32, ra64, rm64, e0, coff,
                                                  hoff);
    else
        feddyn_chunk<DT, 1, false, 0>(sg, row, sflags, n_steps, n_phase1, ra32, rm32, ra64, rm64, e0, coff, hoff);
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
#ifndef FLAME_SLAB_TPW
#define FLAME_SLAB_TPW 2   // slab insert: 4 KiB tiles per workgroup (1-8 within noise, profiles/r03b_slab_sweep.log)
#endif
#ifndef FLAME_SLAB_ST
#define FLAME_SLAB_ST 0    // slab insert: store policy (encoding of FLAME_ST_NT; plain stores measured best)
#endif
constexpr int kSlabTPW = FLAME_SLAB_TPW;
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
        if (kind[j] == 1) st_pol<FLAME_SLAB_ST>(dp[j], v[j]);
}

constexpr int kClientUnroll = FLAME_CU;
constexpr int kClientUnroll16 = FLAME_CU16;
constexpr int kHierUnroll16 = FLAME_HCU16;
constexpr int kOptWGC = FLAME_OPT_WGC;
constexpr int kOptUnroll = FLAME_OPT_CU;
static_assert(kOptWGC >= 1 && kOptWGC <= 32, "FLAME_OPT_WGC: 1..32 chunks per workgroup");
constexpr int kHierLdsUnroll16 = FLAME_HLDS_CU16;
constexpr int kHBL = FLAME_HLDS_BATCH;

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
    const dim3 grid(static_cast<unsigned>((n_chunks + kWGC - 1) / kWGC)), block(kBlock);
    auto cl = reinterpret_cast<const uint64_t*>(clients);
#if FLAME_LO_CU > 0
    // long-lived workgroups over many chunks: two per CU, FLAME_LO_CU loads in flight per lane
    if (n_clients >= FLAME_LO_MIN_CLIENTS && n_chunks >= FLAME_LO_MIN_CHUNKS && kWGC == 1 && FLAME_OCC_LDS == 0) {
        switch (dtype) {
        case FLAME_F32:
            hipLaunchKernelGGL((agg_reduce_kernel<FLAME_F32, FLAME_LO_CU>), grid, block, FLAME_LO_LDS, st, segs, n_segs, cl, n_clients, rates32, rates64, flags, n_chunks);
            return check_launch("flame_agg_reduce");
        case FLAME_BF16:
            hipLaunchKernelGGL((agg_reduce_kernel<FLAME_BF16, FLAME_LO_CU16>), grid, block, FLAME_LO_LDS, st, segs, n_segs, cl, n_clients, rates32, rates64, flags, n_chunks);
            return check_launch("flame_agg_reduce");
        case FLAME_F16:
            hipLaunchKernelGGL((agg_reduce_kernel<FLAME_F16, FLAME_LO_CU16>), grid, block, FLAME_LO_LDS, st, segs, n_segs, cl, n_clients, rates32, rates64, flags, n_chunks);
            return check_launch("flame_agg_reduce");
        default:
            break;      // f64 / integers: the general launch below
        }
    }
#endif
    switch (dtype) {
    case FLAME_F32:
        hipLaunchKernelGGL((agg_reduce_kernel<FLAME_F32, kClientUnroll>), grid, block, FLAME_OCC_LDS, st, segs, n_segs, cl, n_clients, rates32, rates64, flags, n_chunks);
        break;
    case FLAME_BF16:
        hipLaunchKernelGGL((agg_reduce_kernel<FLAME_BF16, kClientUnroll16>), grid, block, FLAME_OCC_LDS, st, segs, n_segs, cl, n_clients, rates32, rates64, flags, n_chunks);
        break;
    case FLAME_F16:
        hipLaunchKernelGGL((agg_reduce_kernel<FLAME_F16, kClientUnroll16>), grid, block, FLAME_OCC_LDS, st, segs, n_segs, cl, n_clients, rates32, rates64, flags, n_chunks);
        break;
    case FLAME_F64:
        hipLaunchKernelGGL((agg_reduce_kernel<FLAME_F64, kClientUnroll>), grid, block, FLAME_OCC_LDS, st, segs, n_segs, cl, n_clients, rates32, rates64, flags, n_chunks);
        break;
    case FLAME_I64:
        hipLaunchKernelGGL((agg_reduce_kernel<FLAME_I64, 4>), grid, block, FLAME_OCC_LDS, st, segs, n_segs, cl, n_clients, rates32, rates64, flags, n_chunks);
        break;
    case FLAME_I32:
        hipLaunchKernelGGL((agg_reduce_kernel<FLAME_I32, 4>), grid, block, FLAME_OCC_LDS, st, segs, n_segs, cl, n_clients, rates32, rates64, flags, n_chunks);
        break;
    default:
        return set_err(FLAME_ENOTSUP, "flame_agg_reduce: unsupported dtype %d", dtype);
    }
    return check_launch("flame_agg_reduce");
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
    const dim3 grid(static_cast<unsigned>((n_chunks + kWGC - 1) / kWGC)), block(kBlock);
#define FLAME_ARGMETA_LAUNCH(DT, CUV) \
    hipLaunchKernelGGL((agg_reduce_kernel_argmeta<DT, CUV>), grid, block, FLAME_OCC_LDS, st, m, n_segs, n_clients, \
                       oc, o32, o64, flags, n_chunks)
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
    return check_launch("flame_agg_reduce_argmeta");
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
    // FLAME_OPT_WGC chunks per workgroup (outputs held in LDS) for fp32 launches big enough to fill
    // the GPU several times over; one chunk per workgroup otherwise
    const bool multi = kOptWGC > 1 && n_chunks >= 8ll * 256 * kOptWGC;
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
    return check_launch("flame_fedopt_reduce_adapt");
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
    const dim3 grid(static_cast<unsigned>(n_chunks)), block(kBlock);
#define FLAME_OPT_ARGMETA_LAUNCH(DT, CUV)                                                                        \
    switch (variant) {                                                                                           \
    case FLAME_FEDADAM:                                                                                          \
        hipLaunchKernelGGL((fedopt_kernel_argmeta<DT, FLAME_FEDADAM, CUV>), grid, block, 0, st, m, n_segs,        \
                           n_clients, oc, o32, flags, b1, omb1, b2, omb2, eta, tau);                             \
        break;                                                                                                   \
    case FLAME_FEDYOGI:                                                                                          \
        hipLaunchKernelGGL((fedopt_kernel_argmeta<DT, FLAME_FEDYOGI, CUV>), grid, block, 0, st, m, n_segs,        \
                           n_clients, oc, o32, flags, b1, omb1, b2, omb2, eta, tau);                             \
        break;                                                                                                   \
    default:                                                                                                     \
        hipLaunchKernelGGL((fedopt_kernel_argmeta<DT, FLAME_FEDADAGRAD, CUV>), grid, block, 0, st, m, n_segs,     \
                           n_clients, oc, o32, flags, b1, omb1, b2, omb2, eta, tau);                             \
        break;                                                                                                   \
    }
    switch (dtype) {
    case FLAME_F32: FLAME_OPT_ARGMETA_LAUNCH(FLAME_F32, kClientUnroll) break;
    case FLAME_BF16: FLAME_OPT_ARGMETA_LAUNCH(FLAME_BF16, kClientUnroll16) break;
    case FLAME_F16: FLAME_OPT_ARGMETA_LAUNCH(FLAME_F16, kClientUnroll16) break;
    default:
        return set_err(FLAME_ENOTSUP, "flame_fedopt_reduce_adapt_argmeta: dtype %d not supported (f32, bf16, f16)", dtype);
    }
#undef FLAME_OPT_ARGMETA_LAUNCH
    return check_launch("flame_fedopt_reduce_adapt_argmeta");
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
    return check_launch("flame_fedbuff_scale_add");
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
#define FLAME_HIER_LAUNCH1(DT, CUV, HB, HL)                                                                    \
    if (sync)                                                                                                  \
        hipLaunchKernelGGL((hier_fedbuff_kernel<DT, CUV, true, HB, HL>), grid, block, FLAME_OCC_LDS, st, segs, n_segs, \
                           n_mids, n_clients, w, d, cl, mid_rates, mid_goal, top_rates, top_goal, flags);      \
    else                                                                                                       \
        hipLaunchKernelGGL((hier_fedbuff_kernel<DT, CUV, false, HB, HL>), grid, block, FLAME_OCC_LDS, st, segs, n_segs, \
                           n_mids, n_clients, w, d, cl, mid_rates, mid_goal, top_rates, top_goal, flags);
    // many middles (config 5: 64 per GPU): LDS-held store groups; a few (a single FedBuff's fused
    // scale_add, small hierarchies): register groups, no LDS, full occupancy
    // one middle over a long launch (a FedBuff aggregator's fused scale_add / a middle's scale_add +
    // delta over >= 64 queued arrivals): fewer workgroups per CU, fewer loads in flight -- fp32 2 per
    // CU unroll 3, 16-bit 3 per CU unroll 3 (64 x 25M: 1.058 -> 0.989 ms fp32, 0.533 -> 0.509 ms bf16;
    // tools/fedbuff_sweep.py, profiles/r03zv_fedbuff_*.log); FLAME_HLO=0 turns it off
#define FLAME_HIER_LO(DT, LDS)                                                                                   \
    hipLaunchKernelGGL((hier_fedbuff_kernel<DT, 3, false, kHB, false>), grid, block, LDS, st, segs, n_segs,     \
                       n_mids, n_clients, w, d, cl, mid_rates, mid_goal, top_rates, top_goal, flags);
#define FLAME_HIER_LAUNCH(DT, CUV, CUL)                                                                        \
    if (FLAME_HLDS && n_mids >= FLAME_HLDS_MIN_MIDS) { FLAME_HIER_LAUNCH1(DT, CUL, kHBL, true) }             \
    else if (FLAME_HLO && !sync && n_mids == 1 && n_clients >= 64 && n_chunks >= 4096 && FLAME_OCC_LDS == 0) {  \
        FLAME_HIER_LO(DT, (DT == FLAME_F32 ? 65536 : 53248))                                                    \
    } else { FLAME_HIER_LAUNCH1(DT, CUV, kHB, false) }
    const bool sync = (flags & FLAME_HIER_SYNC) != 0;
    switch (dtype) {
    case FLAME_F32: FLAME_HIER_LAUNCH(FLAME_F32, kClientUnroll, kClientUnroll) break;
    case FLAME_BF16: FLAME_HIER_LAUNCH(FLAME_BF16, kHierUnroll16, kHierLdsUnroll16) break;
    case FLAME_F16: FLAME_HIER_LAUNCH(FLAME_F16, kHierUnroll16, kHierLdsUnroll16) break;
#undef FLAME_HIER_LAUNCH1
#undef FLAME_HIER_LAUNCH
#undef FLAME_HIER_LO
    default:
        return set_err(FLAME_ENOTSUP, "flame_hier_fedbuff: dtype %d not supported (f32, bf16, f16)", dtype);
    }
    return check_launch("flame_hier_fedbuff");
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
#define FLAME_HIER_ARG_LAUNCH(DT, CUV)                                                                          \
    if (sync)                                                                                                  \
        hipLaunchKernelGGL((hier_fedbuff_kernel_argmeta<DT, CUV, true>), grid, block, FLAME_OCC_LDS, st, m, n_segs, \
                           n_mids, n_clients, ow, od, oc, orr, og, ot, top_goal, flags);                      \
    else                                                                                                       \
        hipLaunchKernelGGL((hier_fedbuff_kernel_argmeta<DT, CUV, false>), grid, block, FLAME_OCC_LDS, st, m, n_segs, \
                           n_mids, n_clients, ow, od, oc, orr, og, ot, top_goal, flags);
    switch (dtype) {
    case FLAME_F32: FLAME_HIER_ARG_LAUNCH(FLAME_F32, kClientUnroll) break;
    case FLAME_BF16: FLAME_HIER_ARG_LAUNCH(FLAME_BF16, kHierUnroll16) break;
    case FLAME_F16: FLAME_HIER_ARG_LAUNCH(FLAME_F16, kHierUnroll16) break;
#undef FLAME_HIER_ARG_LAUNCH
    default:
        return set_err(FLAME_ENOTSUP, "flame_hier_fedbuff_argmeta: dtype %d not supported (f32, bf16, f16)", dtype);
    }
    return check_launch("flame_hier_fedbuff_argmeta");
}

int flame_hier_resident_per_cu(int dtype, unsigned flags, int32_t n_mids) {
    if (n_mids < 1) return -set_err(FLAME_EINVAL, "flame_hier_resident_per_cu: n_mids < 1");
    const bool sync = (flags & FLAME_HIER_SYNC) != 0;
    const bool lds = FLAME_HLDS && n_mids >= FLAME_HLDS_MIN_MIDS;
    const void* f = nullptr;
    // the instantiation FLAME_HIER_LAUNCH in flame_hier_fedbuff picks for these arguments
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
    const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, f, kBlock, FLAME_OCC_LDS);
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
        hipLaunchKernelGGL((feddyn_kernel<FLAME_F32, FLAME_DYN_CU>), grid, block, FLAME_DYN_OCC_LDS, st, segs, n_segs, sp, step_flags, n_steps,
                           n_phase1, ra32, rm32, rate_avg, rate_mean);
        break;
    case FLAME_BF16:
        hipLaunchKernelGGL((feddyn_kernel<FLAME_BF16, FLAME_DYN_CU>), grid, block, FLAME_DYN_OCC_LDS, st, segs, n_segs, sp, step_flags, n_steps,
                           n_phase1, ra32, rm32, rate_avg, rate_mean);
        break;
    case FLAME_F16:
        hipLaunchKernelGGL((feddyn_kernel<FLAME_F16, FLAME_DYN_CU>), grid, block, FLAME_DYN_OCC_LDS, st, segs, n_segs, sp, step_flags, n_steps,
                           n_phase1, ra32, rm32, rate_avg, rate_mean);
        break;
    case FLAME_F64:
        hipLaunchKernelGGL((feddyn_kernel<FLAME_F64, FLAME_DYN_CU>), grid, block, FLAME_DYN_OCC_LDS, st, segs, n_segs, sp, step_flags, n_steps,
                           n_phase1, ra32, rm32, rate_avg, rate_mean);
        break;
    default:
        return set_err(FLAME_ENOTSUP, "flame_feddyn_round: dtype %d not supported (f32, bf16, f16, f64)", dtype);
    }
    return check_launch("flame_feddyn_round");
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

#if FLAME_HTIME
// Diagnostic builds only: where the hierarchy kernel writes its timestamps (NULL = nowhere).
int flame_sweep_htime(void* buf, int32_t slots) {
    uint64_t* p = static_cast<uint64_t*>(buf);
    hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_htime), &p, sizeof(p));
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_htime_slots), &slots, sizeof(slots));
    if (e != hipSuccess) return set_err(FLAME_EHIP, "flame_sweep_htime: %s", hipGetErrorString(e));
    return FLAME_OK;
}
#endif

// The product library's launch-branch counters are not kept in sweep builds (the same symbols,
// so flame_amd._native binds a sweep build too): no branches.
int32_t flame_launch_branches(void) { return 0; }
const char* flame_launch_branch_name(int32_t) { return nullptr; }
int64_t flame_launch_branch_count(int32_t) { return -1; }

}  // extern "C"
