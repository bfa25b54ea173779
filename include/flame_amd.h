/*
 * flame_amd.h -- C ABI of the MI355X-native server-side aggregation path.
 *
 * Drop-in boundary for cisco-open/flame's lib/python data plane.  Each entry
 * point replaces one PyTorch op sequence in the reference (paths relative to
 * /root/reference/lib/python/flame/):
 *
 *   flame_agg_reduce            optimizer/fedavg.py:79-104   (FedAvg.do client loop +
 *                                                             _aggregate_pytorch)
 *                               optimizer/fedbuff.py:89-97,136-157 (FedBuff.do loop +
 *                                                             _aggregate_pytorch)
 *   flame_fedopt_reduce_adapt   optimizer/fedopt.py:80-90,102-129 (FedAvg.do + _adapt_pytorch)
 *                               + fedadam.py:33-35 / fedyogi.py:34-36 / fedadagrad.py:33-35
 *   flame_fedbuff_scale_add     optimizer/fedbuff.py:101-127 (scale_add_agg_weights), fused with
 *                               common/util.py:152-159 (delta_weights_pytorch) as used by
 *                               mode/horizontal/asyncfl/middle_aggregator.py:221-226,246
 *   flame_hier_fedbuff          a node's co-located two-level FedBuff hierarchy in one pass
 *                               (FLAME_HIER_SYNC: the synchronous FedAvg hierarchy,
 *                               syncfl/middle_aggregator.py:163-229 -> syncfl/top_aggregator.py:122-176):
 *                               per middle optimizer/fedbuff.py:89-97,136-157 (None-start
 *                               arrivals) + :101-127 (scale_add) + the delta of
 *                               mode/horizontal/asyncfl/middle_aggregator.py:221-226,246,
 *                               fed to the top's FedBuff (asyncfl/top_aggregator.py:85-109)
 *   flame_feddyn_round          optimizer/feddyn.py:90-113,125-139 (FedDyn.do: add_to_hist,
 *                               FedAvg with rate 1/len(cache), mean of the histories, cld_model)
 *   flame_elementwise           the same statements for the keys the fused kernels do not take
 *                               (int / mixed-dtype / fp64 keys): optimizer/fedopt.py:102-129,
 *                               scaffold.py:141-150, feddyn.py:90-113,125-139
 *   flame_synth_fill            (bench/test plumbing: counter-based synthetic updates)
 *   flame_hier_resident_per_cu  (no reference counterpart: occupancy query the parameter
 *                               shard uses to size its waves, flame_amd/shard.py)
 *
 * Conventions
 *   - All pointers passed to the compute entry points are DEVICE pointers
 *     (HBM of the current HIP device) unless stated otherwise; `stream` is a
 *     hipStream_t (NULL = default stream).  Calls are asynchronous on `stream`.
 *   - Per element, clients are combined strictly in the order given (the
 *     reference's cache.iterkeys() order); each reference op is one IEEE
 *     round-to-nearest-even rounding in the tensor's dtype (no FMA), so results
 *     are bit-identical to the reference's torch-CPU arithmetic for
 *     FedAvg/FedBuff.  Only FedOPT's sqrt differs (torch-CPU's fp32 sqrt is not
 *     correctly rounded; ours is).
 *   - Return value: FLAME_OK (0) or a nonzero FLAME_E* status; the message is
 *     available from flame_last_error() (thread-local).  Nothing aborts.
 */
#ifndef FLAME_AMD_H
#define FLAME_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FLAME_ABI_VERSION 1

/* status codes */
#define FLAME_OK 0
#define FLAME_EINVAL 1   /* bad argument (message in flame_last_error) */
#define FLAME_EHIP 2     /* HIP runtime error (launch / device) */
#define FLAME_ENOTSUP 3  /* dtype / variant not supported by this entry point */

/* element types (torch dtypes of the reference state_dict tensors) */
#define FLAME_F32 0
#define FLAME_BF16 1
#define FLAME_F16 2
#define FLAME_F64 3
#define FLAME_I64 4
#define FLAME_I32 5

/* flame_agg_reduce flags */
#define FLAME_AGG_INIT_FIRST 1u  /* no base: acc = tmp(client 0) (fedbuff.py:139-140,154-155) */
#define FLAME_AGG_SEG_RATES 2u   /* rates are [n_segs][n_clients]: one rate row per segment
                                    (independent reductions -- e.g. the middle aggregators of
                                    a node, asyncfl/middle_aggregator.py:164-256 -- in one launch) */
#define FLAME_AGG_XCD_MAP 4u     /* workgroups take chunks XCD by XCD (each of the 8 XCDs, which get
                                    workgroups round-robin, streams one contiguous eighth of the
                                    chunks): faster when every client is its own tensor (rows),
                                    slower for a tiled UpdateSlab; results are identical */

/* flame_fedopt_reduce_adapt variants and flags */
#define FLAME_FEDADAM 0
#define FLAME_FEDYOGI 1
#define FLAME_FEDADAGRAD 2
#define FLAME_OPT_STATE_ZERO 1u  /* m_t, v_t were None: treat as zeros, do not read (fedopt.py:108-122) */
#define FLAME_OPT_XCD_MAP 2u     /* as FLAME_AGG_XCD_MAP, for flame_fedopt_reduce_adapt */

/* per-segment flag (flame_segment.flags) */
#define FLAME_SEG_UNALIGNED 1    /* some pointer of this segment is not 16-byte aligned */
#define FLAME_SEG_CUR_IS_AVG 2   /* flame_fedopt_reduce_adapt: `cur` IS the FedAvg result (the eager
                                    caller's current_weights alias base_weights after the round-1
                                    passthrough, eager_syncfl/top_aggregator.py:42,75 +
                                    fedopt.py:87-88): cur takes the reduced value, d = avg - avg;
                                    seg.cur is not read */

/*
 * One contiguous run of elements (typically one state_dict tensor, or one
 * dtype group of a flattened model).  Field roles by entry point:
 *
 *                 flame_agg_reduce     flame_fedopt_reduce_adapt   flame_fedbuff_scale_add
 *   out           aggregate (out)      FedAvg result (out, opt.)   base weights (in/out)
 *   in            base (in; may ==out) base weights (in)           agg_goal_weights (in)
 *   cur           -                    current weights (in)        -
 *   cur_out       -                    new current weights (out)   delta = new-old (out, opt.)
 *   m, v          -                    m_t, v_t (in/out)           -
 *
 * chunk_begin is the prefix sum over previous segments of
 * ceil(numel / flame_chunk_elems(dtype)); the grid covers n_chunks chunks.
 * client_tile_stride (reduce entry points only): 0 = every client's data for
 * the segment is contiguous; otherwise client data is TILED -- chunk c of a
 * client starts client_tile_stride bytes after chunk c-1 (e.g. a [chunks][N][chunk]
 * slab, where one workgroup reads one contiguous N x chunk region).
 * The table lives in device memory.
 */
typedef struct flame_segment {
    void *out;
    const void *in;
    const void *cur;
    void *cur_out;
    void *m;
    void *v;
    int64_t numel;
    int64_t chunk_begin;
    int64_t flags;
    int64_t client_tile_stride;
} flame_segment;

/* Library info. */
int flame_abi_version(void);
const char *flame_last_error(void);
/* Elements one workgroup covers per segment chunk for `dtype` (0 if invalid). */
int64_t flame_chunk_elems(int dtype);
/* Elements per chunk for the elementwise scale-add kernel. */
int64_t flame_scale_add_chunk_elems(int dtype);

/*
 * Weighted client reduction (FedAvg / FedBuff accumulate).
 *   clients : device array [n_segs][n_clients] of device pointers; row s holds,
 *             in iteration order, each client's data for segment s.
 *   rates32 : device [n_clients] fp32 rates (float(count/total) or
 *             float(1/sqrt(1+version-tres.version))), used for every dtype but f64.
 *   rates64 : device [n_clients] fp64 rates, used for FLAME_F64 (may be NULL otherwise).
 *             With FLAME_AGG_SEG_RATES both are [n_segs][n_clients] and segment s uses row s.
 * Per element e of each segment:
 *   acc = in[e] (or tmp_0 with FLAME_AGG_INIT_FIRST);
 *   for i: tmp = round(v_i[e] * rate_i) (ints: trunc(float(v)*rate)); acc = round(acc + tmp)
 *   out[e] = acc.
 */
int flame_agg_reduce(int dtype, unsigned flags, const flame_segment *segs, int32_t n_segs,
                     int64_t n_chunks, const void *const *clients, int32_t n_clients,
                     const float *rates32, const double *rates64, void *stream);

/*
 * flame_agg_reduce for small launches: the same metadata block (segments, then the client
 * pointer table and the rates, at byte offsets off_clients / off_r32 / off_r64 -- pass -1 for
 * the rate array the dtype does not use) is passed from HOST memory and travels to the GPU as
 * a kernel argument, so no H2D copy (a blit kernel on gfx950, ≈15 µs of GPU timeline per
 * launch) precedes the reduction.  meta_bytes <= flame_agg_argmeta_max_bytes() (3,584).
 * Semantics, flags and dtypes as flame_agg_reduce; the client and segment pointers inside
 * the block are device pointers as there.
 */
int flame_agg_reduce_argmeta(int dtype, unsigned flags, const void *host_meta, int64_t meta_bytes,
                             int32_t n_segs, int64_t n_chunks, int32_t n_clients, int64_t off_clients,
                             int64_t off_r32, int64_t off_r64, void *stream);
int64_t flame_agg_argmeta_max_bytes(void);

/*
 * Fused FedAvg + FedOPT adaptive step (dtype FLAME_F32, FLAME_BF16 or FLAME_F16; base,
 * cur, m, v, outputs and clients all of that dtype).  After the reduction above (avg kept
 * in registers, optionally written to seg.out), per element, every op rounded in dtype:
 *   d = avg - cur; m = b1*m + omb1*d;
 *   Adam: v = b2*v + omb2*(d*d);  Yogi: v = v - omb2*(d*d)*sign(v - d*d);  AdaGrad: v = v + d*d
 *   cur_out = cur + (eta*m) / (sqrt(v) + tau)
 * (a segment flagged FLAME_SEG_CUR_IS_AVG takes cur = avg, as the reference does when
 * current_weights and base_weights are one object).
 * Scalars are the roundings torch applies to the Python floats: b1 = f32(beta_1),
 * omb1 = f32(1 - beta_1), b2 = f32(beta_2), omb2 = f32(1 - beta_2), eta = f32(eta),
 * tau = f32(tau) for fp32 but dtype(tau) for bf16/fp16 (torch-CPU rounds a scalar to a
 * reduced-precision tensor's dtype before + / -).
 */
int flame_fedopt_reduce_adapt(int dtype, int variant, unsigned flags, const flame_segment *segs,
                              int32_t n_segs, int64_t n_chunks, const void *const *clients,
                              int32_t n_clients, const float *rates32, float b1, float omb1,
                              float b2, float omb2, float eta, float tau, void *stream);

/*
 * Eager FedOPT chain (FLAME_F32, FLAME_BF16 or FLAME_F16; every tensor of a segment of that
 * dtype, scalars as for flame_fedopt_reduce_adapt): the eager top aggregator's per-arrival do() calls
 * (eager_syncfl/top_aggregator.py:36-90, fedavg.py:93-104 then fedopt.py:102-129), queued and
 * run in one pass.  Per element, for each client i in order: base = base + round(w_i * r_i);
 * where step_end[i] != 0 (device array, one byte per client; client i closes a do() call) the
 * adaptive step of flame_fedopt_reduce_adapt with avg = base and the running current (the
 * first step of a segment flagged FLAME_SEG_CUR_IS_AVG takes cur = base).  Writes base to
 * seg.out, m and v in place, the final current to seg.cur_out (seg.cur is read unless the
 * segment is flagged).  FLAME_OPT_STATE_ZERO: m, v start as zeros and are not read.  Bitwise
 * equal to one flame_fedopt_reduce_adapt launch per do() call.  Replaces, per round,
 * optimizer/fedopt.py:80-90,102-129 as the eager role calls it.
 */
int flame_fedopt_chain(int dtype, int variant, unsigned flags, const flame_segment *segs, int32_t n_segs,
                       int64_t n_chunks, const void *const *clients, int32_t n_clients,
                       const float *rates32, const uint8_t *step_end, float b1, float omb1, float b2,
                       float omb2, float eta, float tau, void *stream);

/*
 * flame_fedopt_reduce_adapt with its metadata block (segments, then the [n_segs][n_clients]
 * client table at byte offset off_clients, then the fp32 rates at off_r32; at most
 * flame_agg_argmeta_max_bytes() bytes, host memory) passed as a kernel argument: no
 * device table and no H2D copy before the launch.  Small rounds only (e.g. flame's MNIST
 * model x a few trainers).  Replaces the same reference code as flame_fedopt_reduce_adapt
 * (optimizer/fedopt.py:80-90,102-129).  FLAME_EINVAL if a table lies outside the block.
 */
int flame_fedopt_reduce_adapt_argmeta(int dtype, int variant, unsigned flags, const void *host_meta,
                                      int64_t meta_bytes, int32_t n_segs, int64_t n_chunks,
                                      int32_t n_clients, int64_t off_clients, int64_t off_r32,
                                      float b1, float omb1, float b2, float omb2, float eta,
                                      float tau, void *stream);

/*
 * FedBuff scale-add: out[e] = round(out[e] + round(in[e] / goal)); if seg.cur_out
 * is non-NULL also cur_out[e] = round(new - old) (the middle aggregator's delta).
 * Float dtypes only (the reference raises for integer tensors).
 */
int flame_fedbuff_scale_add(int dtype, const flame_segment *segs, int32_t n_segs,
                            int64_t n_chunks, int64_t goal, void *stream);

/* flame_hier_fedbuff flags */
#define FLAME_HIER_TOP_ACCUM 1u  /* the top aggregate exists (not None): start from seg.top_agg_in */
#define FLAME_HIER_TOP_APPLY 2u  /* finish with the top's scale-add into seg.top_w */
#define FLAME_HIER_MID_READONLY 4u  /* do not write w_m' back: the middles' weights are only the
                                      base of their deltas (the async middle role replaces them with
                                      the top's model at its next fetch,
                                      asyncfl/middle_aggregator.py:119-120); mid_w may then alias */
#define FLAME_HIER_SYNC 8u   /* the synchronous hierarchy (syncfl/middle_aggregator.py:163-229 feeding
                                syncfl/top_aggregator.py:122-176): per middle FedAvg from its weights,
                                a = w_m + tmp(c_{m,0}, r_{m,0}) + ..., w_m' = a, d_m = w_m' - w_m; the top
                                is a FedAvg from its weights: top = top_agg_in + tmp(d_m, top_rates[m]) in
                                order.  Needs FLAME_HIER_TOP_ACCUM, excludes FLAME_HIER_TOP_APPLY; mid_goal
                                is not read (any values) */

/* One contiguous run of elements of the hierarchy (one state_dict tensor). */
typedef struct flame_hier_segment {
    void *top_w;              /* top model weights, in/out (FLAME_HIER_TOP_APPLY) */
    const void *top_agg_in;   /* top aggregate before this batch (FLAME_HIER_TOP_ACCUM) */
    void *top_agg_out;        /* top aggregate after this batch (NULL = not stored; may == top_agg_in) */
    int64_t numel;
    int64_t chunk_begin;      /* prefix sum of ceil(numel / flame_chunk_elems(dtype)) */
    int64_t flags;            /* FLAME_SEG_UNALIGNED */
    int64_t client_tile_stride;  /* as flame_segment.client_tile_stride, shared by every arrival */
    int64_t mid_tile_stride;  /* bytes between consecutive chunks of one middle's weights (0 = each
                                 middle's weights contiguous); nonzero: every middle's weights are
                                 tiled like the arrivals (slots of one flame_amd UpdateSlab), so a
                                 chunk's middle weights form one contiguous [n_mids][chunk] block */
} flame_hier_segment;

/*
 * Co-located two-level FedBuff hierarchy (LIFL-style: n_mids middle aggregators on this
 * GPU feeding one top aggregator), one launch.  Per element, for m = 0 .. n_mids-1 (the
 * order the top receives the middles' deltas), every op rounded in dtype:
 *   a   = tmp(c_{m,0}, r_{m,0}); a = a + tmp(c_{m,i}, r_{m,i}) for i >= 1     (None-start FedBuff)
 *   w_m' = w_m + a / mid_goal[m];  d_m = w_m' - w_m;  w_m := w_m'          (scale_add + delta)
 *   top = tmp(d_0, top_rates[0]) (or top_agg_in + ...), top = top + tmp(d_m, top_rates[m])
 * then top_agg_out = top and, with FLAME_HIER_TOP_APPLY, top_w = top_w + top / top_goal.
 * tmp(v, r) = round(v * r).  Bit-identical to flame_agg_reduce (INIT_FIRST) per middle +
 * flame_fedbuff_scale_add with delta + one flame_agg_reduce per delta on the top aggregate +
 * flame_fedbuff_scale_add; the middle aggregates never reach HBM.
 *   mid_w     : device [n_segs][n_mids] pointers to each middle's weights (in/out; in only with
 *               FLAME_HIER_MID_READONLY)
 *   mid_delta : device [n_segs][n_mids] pointers for the deltas (NULL table or NULL entries:
 *               not stored)
 *   clients   : device [n_segs][n_mids][n_clients] arrival pointers, arrival order per middle
 *   mid_rates : device [n_mids][n_clients] fp32 staleness rates float(1/sqrt(1+version-v))
 *   mid_goal  : device [n_mids] float(agg_goal) of each middle; top_rates: device [n_mids]
 * dtype FLAME_F32, FLAME_BF16 or FLAME_F16.
 * With n_mids = 1, top_agg_out = NULL and no flags this is a single FedBuff aggregator's
 * scale_add (optimizer/fedbuff.py:101-127) applied straight from its queued arrivals
 * (fedbuff.py:89-97,136-157) -- the aggregate is never stored (the async top's round,
 * asyncfl/top_aggregator.py:85-110).
 */
int flame_hier_fedbuff(int dtype, unsigned flags, const flame_hier_segment *segs, int32_t n_segs,
                       int64_t n_chunks, int32_t n_mids, int32_t n_clients, const void *const *mid_w,
                       const void *const *mid_delta, const void *const *clients,
                       const float *mid_rates, const float *mid_goal, const float *top_rates,
                       float top_goal, void *stream);

/* flame_feddyn_round step flags */
#define FLAME_DYN_W 1u      /* the step has an arrival w (steps[..][0]) */
#define FLAME_DYN_AVG 2u    /* avg = avg + tmp(w, rate_avg)            (needs W) */
#define FLAME_DYN_HIN 4u    /* load the history h (steps[..][1]) */
#define FLAME_DYN_HOUT 8u   /* h' = HIN ? h + w : w, stored to steps[..][2] (needs W) */
#define FLAME_DYN_MEAN 16u  /* mean = mean + tmp(HOUT ? h' : h, rate_mean) (needs HIN or HOUT) */
/* One contiguous run of elements of a FedDyn round (one state_dict tensor). */
typedef struct flame_dyn_segment {
    void *out;                   /* the average (may == in) */
    const void *in;              /* base weights: the FedAvg start (deepcopy of cld_model) */
    void *cld;                   /* cld_model = avg + mean history (out) */
    int64_t numel;
    int64_t chunk_begin;         /* prefix sum of ceil(numel / flame_chunk_elems(dtype)) */
    int64_t flags;               /* FLAME_SEG_UNALIGNED */
    int64_t client_tile_stride;  /* arrivals: as flame_segment.client_tile_stride */
    int64_t hist_tile_stride;    /* histories: 0 = contiguous, else bytes between their chunks */
} flame_dyn_segment;
/*
 * One FedDyn server round (optimizer/feddyn.py:90-113 do() + :125-139 add_to_hist) in one
 * launch, per dtype.  steps: device [n_segs][n_steps][3] pointers (w, h_in,
 * h_out) per segment; step_flags: device [n_steps].  Per element, steps run in order with
 * mean starting at +0 (`0.0 + Σ rate*h`); every op rounds in dtype as torch-CPU does, so the
 * result is bit-identical to the reference's op sequence when the program lists the
 * arrivals in cache.iterkeys() order (AVG) and the histories in local_param_dict order
 * (MEAN).  Steps [n_phase1, n_steps) start after every earlier step's store, so they may
 * re-read a history written by a phase-1 step; within a phase no step may read another
 * step's output.  rate_avg = 1/len(cache), rate_mean = 1/len(local_param_dict) (rounded to
 * fp32 for f32/bf16/f16).  dtype FLAME_F32, FLAME_BF16, FLAME_F16 or FLAME_F64.
 */
int flame_feddyn_round(int dtype, const flame_dyn_segment *segs, int32_t n_segs, int64_t n_chunks,
                       const void *const *steps, const uint32_t *step_flags, int32_t n_steps,
                       int32_t n_phase1, double rate_avg, double rate_mean, void *stream);
/*
 * flame_elementwise: one elementwise program -- a short typed op sequence, the reference's
 * own torch statements for the keys the fused kernels do not take (int buffers such as
 * num_batches_tracked, mixed-dtype keys, fp64 / int8 / uint8 / int16 tensors):
 *   optimizer/fedopt.py:102-129 + fedadam.py:33-35 / fedyogi.py:34-36 / fedadagrad.py:33-35
 *     (FedOPT's adaptive step: d, m, v, sqrt(v) + tau, the quotient, current + ...),
 *   optimizer/scaffold.py:141-150 (c += (w * rate).to(c.dtype) for a control of another dtype),
 *   optimizer/feddyn.py:90-113,125-139 (the history / mean / cld statements of mixed keys).
 * flame_amd/elementwise.py records the statements on lazy tensors and takes every result dtype
 * from torch's own promotion (the statements run on meta tensors of the same shapes), so a
 * program only ever computes what torch-CPU would: an op whose operands are cast (FLAME_EW_CAST)
 * to its result dtype first, then
 *   fp32 / fp64: one IEEE round-to-nearest-even op (sqrt / divide correctly rounded);
 *   bf16 / fp16: the op in fp32 on the widened operands, rounded once to the dtype; a scalar
 *     is used in fp32 by MUL_S and rounded to the dtype first by ADD_S (torch-CPU's behaviour);
 *   integers: two's-complement arithmetic wrapped to the dtype's width (bool: + is a logical
 *     or, * a logical and, - is refused as torch refuses it).
 * Per element i of [0, numel): registers r[0..FLAME_EW_MAX_REGS) start undefined; ops run in
 * order.  prog (n_ops <= FLAME_EW_MAX_OPS) and bufs (n_bufs <= FLAME_EW_MAX_BUFS) are HOST
 * arrays, copied into the launch; every buffer is a contiguous DEVICE array of numel elements.
 */
#define FLAME_U8 6     /* element types only flame_elementwise takes */
#define FLAME_I8 7
#define FLAME_I16 8
#define FLAME_BOOL 9
#define FLAME_EW_LOAD 0    /* r[dst] = bufs[a][i], read as dtype */
#define FLAME_EW_STORE 1   /* bufs[a][i] = r[b], written as dtype (= r[b]'s dtype) */
#define FLAME_EW_ZERO 2    /* r[dst] = 0 (torch.zeros_like) */
#define FLAME_EW_CAST 3    /* r[dst] = r[a] (dtype b) as dtype: int -> float RNE (via fp32 for
                              bf16 / fp16, as c10 converts), float -> narrower float RNE (fp64 ->
                              bf16 / fp16 via fp32), float -> int toward zero, int -> int wrapped,
                              to bool: != 0 */
#define FLAME_EW_ADD 4     /* r[dst] = r[a] + r[b] (both already dtype) */
#define FLAME_EW_SUB 5     /* r[a] - r[b] */
#define FLAME_EW_MUL 6     /* r[a] * r[b] */
#define FLAME_EW_DIV 7     /* r[a] / r[b] (float dtype: torch's true division) */
#define FLAME_EW_ADD_S 8   /* r[a] + scalar */
#define FLAME_EW_MUL_S 9   /* r[a] * scalar */
#define FLAME_EW_SQUARE 10 /* r[a] ** 2 */
#define FLAME_EW_SIGN 11   /* torch.sign (NaN and -0 -> +0 for floats) */
#define FLAME_EW_SQRT 12   /* torch.sqrt (float dtype) */
#define FLAME_EW_MAX_OPS 64
#define FLAME_EW_MAX_REGS 32
#define FLAME_EW_MAX_BUFS 16
typedef struct flame_ew_op {
    int32_t op;      /* FLAME_EW_* */
    int32_t dtype;   /* the result's element type (LOAD / STORE: the buffer's) */
    int32_t dst;     /* register written */
    int32_t a;       /* register read (LOAD / STORE: the buffer index) */
    int32_t b;       /* second register read (STORE: the register stored; CAST: r[a]'s dtype) */
    int32_t pad;
    double scalar;   /* ADD_S / MUL_S: the Python scalar */
} flame_ew_op;
int flame_elementwise(const flame_ew_op *prog, int32_t n_ops, void *const *bufs, int32_t n_bufs,
                      int64_t numel, void *stream);
/*
 * The same program over several segments in one launch (e.g. a ResNet's BatchNorm
 * num_batches_tracked keys, which share one program): table = DEVICE [n_segs][n_bufs] buffer
 * pointers, seg_end = DEVICE [n_segs] inclusive prefix sums of the segments' element counts,
 * numel = seg_end[n_segs - 1].  prog is a HOST array as above.
 */
int flame_elementwise_segments(const flame_ew_op *prog, int32_t n_ops, void *const *table, int32_t n_bufs,
                               const int64_t *seg_end, int32_t n_segs, int64_t numel, void *stream);

/*
 * flame_hier_fedbuff for small launches: the metadata block (segments, then the mid_w,
 * mid_delta, client, mid_rates, mid_goal and top_rates tables at the given byte offsets;
 * off_mid_delta = -1 for none) is passed from HOST memory as a kernel argument instead of
 * being copied to the device first.  meta_bytes <= flame_agg_argmeta_max_bytes().
 */
int flame_hier_fedbuff_argmeta(int dtype, unsigned flags, const void *host_meta, int64_t meta_bytes,
                               int32_t n_segs, int64_t n_chunks, int32_t n_mids, int32_t n_clients,
                               int64_t off_mid_w, int64_t off_mid_delta, int64_t off_clients,
                               int64_t off_mid_rates, int64_t off_mid_goal, int64_t off_top_rates,
                               float top_goal, void *stream);

/*
 * Workgroups of the flame_hier_fedbuff launch for (dtype, n_mids, FLAME_HIER_SYNC in flags)
 * that stay resident per CU at once (hipOccupancyMaxActiveBlocksPerMultiprocessor on the
 * instantiation flame_hier_fedbuff would pick).  Its workgroups are long-lived (a chunk's
 * every arrival), so a launch of chunks not a multiple of (this x CUs) ends in a partly
 * filled last round of workgroups; flame_amd.shard sizes its waves with it.  Returns the
 * count (>= 1) or a negative FLAME_E* status (host-side query, no launch).
 */
int flame_hier_resident_per_cu(int dtype, unsigned flags, int32_t n_mids);

/*
 * Host buffers the kernels read zero-copy over PCIe (ingest; flame_amd/ingest.py).
 *   flame_host_register:   page-lock + map an existing host range (e.g. a received
 *                          channel payload or the LIFL shared-memory segment,
 *                          lib/python/flame/backend/shm.py:386-403) for device access.
 *   flame_host_unregister: undo it.
 *   flame_host_device_pointer: device address of a pinned / registered host address
 *                          (hipHostMalloc'd memory maps to itself).
 */
int flame_host_register(void *host, uint64_t nbytes);
int flame_host_unregister(void *host);
int flame_host_device_pointer(void *host, void **device);

/*
 * Fill out[0..numel) with the counter-based generator of flame_amd/synth.py:
 *   value_f32(seed, stream_id, start + j) * scale, rounded RNE to `dtype`
 *   (FLAME_F32 / FLAME_BF16 / FLAME_F16).  `out` is a device pointer.
 */
int flame_synth_fill(int dtype, void *out, int64_t numel, uint64_t seed, uint64_t stream_id,
                     int64_t start, float scale, void *stream);

/*
 * Slab insert: the aggregator role's `self.cache[end] = tres` (mode/horizontal/syncfl/
 * top_aggregator.py:154-156, asyncfl/top_aggregator.py:85-87) into a tiled update slab
 * (flame_amd/slab.py).  Per entry (one state_dict key of one update): the `nbytes`
 * contiguous bytes at `src` are cut into FLAME_TILE_BYTES tiles (one reduction chunk of
 * every dtype, = flame_chunk_elems(dtype) x itemsize) and tile t is written to
 * dst + t * dst_tile_stride; the last tile may be partial (bytes past nbytes untouched).
 * dst must be 16-byte aligned, dst_tile_stride >= FLAME_TILE_BYTES and a multiple of 16
 * when the entry spans more than one tile; src may have any alignment; nbytes == 0 entries
 * are skipped.
 *   flame_slab_write    : ONE kernel launch for up to 89 entries (the table travels as a
 *                         kernel argument, no metadata H2D); src is a device pointer (or a
 *                         mapped pinned-host pointer, read over PCIe).
 *   flame_slab_write_2d : per entry one hipMemcpy2DAsync (pitch = dst_tile_stride) plus one
 *                         hipMemcpyAsync for a ragged tail, on the copy engines; for host
 *                         sources (pinned, registered or pageable).
 * Both are asynchronous on `stream`.
 */
#define FLAME_TILE_BYTES 4096
typedef struct flame_tile_copy {
    const void *src;
    void *dst;
    int64_t nbytes;
    int64_t dst_tile_stride;
} flame_tile_copy;
int flame_slab_write(const flame_tile_copy *table, int32_t n_entries, void *stream);
int flame_slab_write_2d(const flame_tile_copy *table, int32_t n_entries, void *stream);

/*
 * Launch-branch counters (test and audit support; no reference counterpart).  Every
 * host-side branch of the launch entry points above that picks a kernel instantiation
 * (dtype, variant, residency, store-group mode) has an index in [0, flame_launch_branches());
 * each successful launch increments its branch's process-wide counter.
 *   flame_launch_branch_name  : "entry/mode/dtype[/variant]", NULL outside the range
 *   flame_launch_branch_count : launches so far, -1 outside the range
 */
int32_t flame_launch_branches(void);
const char *flame_launch_branch_name(int32_t branch);
int64_t flame_launch_branch_count(int32_t branch);

#ifdef __cplusplus
}
#endif
#endif /* FLAME_AMD_H */
