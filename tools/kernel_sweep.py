#!/usr/bin/env python3
"""Interleaved A/B sweep of compile-time variants of flame_agg_reduce (fp32).

Each variant is a build of the product source (flame_amd/csrc/fedagg.hip) with -DFLAME_T_*
overrides of its tunables, loaded side by side with ctypes;
all run in ONE process on the same device-resident 1024 x 25M slab, rounds
interleaved (cdna_hip_programming.md §5.4 rule 24), outputs checked bitwise
against the first variant.

    python tools/kernel_sweep.py --build          # build variants (here or on the box)
    python tools/kernel_sweep.py --rounds 5       # on the GPU
"""
import argparse
import ctypes
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
VDIR = os.path.join(ROOT, "build", "ab", "variants")   # travels to the GPU box with the tree

# Knobs of the PRODUCT source (flame_amd/csrc/fedagg.hip's FLAME_T_* defaults are the shipped
# kernel).  Variants of rounds 1-4 that were measured no faster and are no longer in the source
# (block size, vectors per lane, pipelining, store policies, buffer loads, FedDyn LDS bursts, ...)
# are recorded in profiles/r0*_sweep*.log and DESIGN.md §4.
VARIANTS = {
    "base": {},
    "cu4": {"FLAME_T_CLIENT_UNROLL": 4},
    "cu16": {"FLAME_T_CLIENT_UNROLL": 16},
    "lo_cu2": {"FLAME_T_LO_UNROLL": 2},
    "lo_cu4": {"FLAME_T_LO_UNROLL": 4},
    "lo_occ3": {"FLAME_T_LO_LDS": 53248},
    "optwgc2": {"FLAME_T_OPT_WGC": 2},
    "optwgc8": {"FLAME_T_OPT_WGC": 8},
    "optcu4": {"FLAME_T_OPT_UNROLL": 4},
    "dyncu2": {"FLAME_T_DYN_UNROLL": 2},
    "dyncu8": {"FLAME_T_DYN_UNROLL": 8},
    "chain_cu8_full": {"FLAME_T_CHAIN_UNROLL": 8, "FLAME_T_CHAIN_LDS": 0},     # round 4's configuration
    "chain_cu4": {"FLAME_T_CHAIN_UNROLL": 4},
    "chain_cu16": {"FLAME_T_CHAIN_UNROLL": 16},
    "chain_occ4": {"FLAME_T_CHAIN_LDS": 40960},     # 4 workgroups per CU
    "chain_occ3": {"FLAME_T_CHAIN_LDS": 53248},
    "chain_occ2": {"FLAME_T_CHAIN_LDS": 65536},
    "chain_cu16_occ3": {"FLAME_T_CHAIN_UNROLL": 16, "FLAME_T_CHAIN_LDS": 53248},
    "chain_cu16_occ4": {"FLAME_T_CHAIN_UNROLL": 16, "FLAME_T_CHAIN_LDS": 40960},
    "chain_cu12_occ3": {"FLAME_T_CHAIN_UNROLL": 12, "FLAME_T_CHAIN_LDS": 53248},
    "chain_cu32": {"FLAME_T_CHAIN_UNROLL": 32},
    "chain_cu24_occ3": {"FLAME_T_CHAIN_UNROLL": 24, "FLAME_T_CHAIN_LDS": 53248},
    # the low-residency reduction's LDS-held output bursts (kLoWGC chunks per workgroup, below
    # kLoBurstMaxClients clients): none, and 8 / 16 / 32 chunks at every client count
    # config 2 (256 clients x 1M fp32, 977 chunks): below the low-residency launch's 4,096 chunks
    "c2_lo": {"FLAME_T_LO_MIN_CHUNKS": 512, "FLAME_T_LO_WGC": 1},
    "c2_lo_occ3": {"FLAME_T_LO_MIN_CHUNKS": 512, "FLAME_T_LO_WGC": 1, "FLAME_T_LO_LDS": 53248},
    "c2_lo_occ4": {"FLAME_T_LO_MIN_CHUNKS": 512, "FLAME_T_LO_WGC": 1, "FLAME_T_LO_LDS": 40960},
    "c2_cu4": {"FLAME_T_CLIENT_UNROLL": 4},
    "c2_cu16": {"FLAME_T_CLIENT_UNROLL": 16},
    "lo_wgc1": {"FLAME_T_LO_WGC": 1},
    "lo_wgc8_all": {"FLAME_T_LO_WGC": 8, "FLAME_T_LO_BURST_MAX_CLIENTS": 1 << 30},
    "lo_wgc16_all": {"FLAME_T_LO_WGC": 16, "FLAME_T_LO_BURST_MAX_CLIENTS": 1 << 30},
    "lo_wgc32_all": {"FLAME_T_LO_WGC": 32, "FLAME_T_LO_BURST_MAX_CLIENTS": 1 << 30},
    # round 6: the round-5 bf16 FedOPT step / Yogi sign (generic per-element code), for the chain A/B
    # (the 16-bit steps' per-element code: bf16 and fp16; lib_r05_step.so was built before the fp16
    # packed step existed, and these defines rebuild the same code)
    "r05_step": {"FLAME_T_BF16_PACKED": 0, "FLAME_T_YOGI_SIGN": 0, "FLAME_T_F16_PACKED": 0},
    "r05_bf16": {"FLAME_T_BF16_PACKED": 0},
    "r05_yogi": {"FLAME_T_YOGI_SIGN": 0},
    # the shipped library with the 16-bit steps on the fp32 step's fast-path admission
    "r06_admit": {"FLAME_T_HALF_ADMIT": 0},
    # the fp16 eager chain on fp32 registers (the step before the packed-fp16 chain body)
    "r06_f16": {"FLAME_T_F16_NATIVE": 0},
}


def build_variants(names):
    from flame_amd import build as B
    os.makedirs(VDIR, exist_ok=True)
    for name in names:
        defs = [f"-D{k}={v}" for k, v in VARIANTS[name].items()]
        out = os.path.join(VDIR, f"lib_{name}.so")
        cmd = [B.hipcc(), *B.HIPCC_FLAGS, *defs, "-o", out, B.SRC]
        subprocess.check_call(cmd)
        print("built", out, flush=True)


def load(name):
    # a name with a "/" is a library path (e.g. build/ab/lib_prev.so)
    L = ctypes.CDLL(os.path.join(ROOT, name) if "/" in name else os.path.join(VDIR, f"lib_{name}.so"))
    vp, i32, i64, u32 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint
    L.flame_chunk_elems.restype = i64
    L.flame_chunk_elems.argtypes = [ctypes.c_int]
    L.flame_agg_reduce.restype = ctypes.c_int
    L.flame_agg_reduce.argtypes = [ctypes.c_int, u32, vp, i32, i64, vp, i32, vp, vp, vp]
    L.flame_last_error.restype = ctypes.c_char_p
    L.flame_fedopt_reduce_adapt.restype = ctypes.c_int
    L.flame_fedopt_reduce_adapt.argtypes = [ctypes.c_int, ctypes.c_int, u32, vp, i32, i64, vp, i32, vp] + \
        [ctypes.c_float] * 6 + [vp]
    return L


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--variants", default=",".join(VARIANTS))
    ap.add_argument("--clients", type=int, default=1024)
    ap.add_argument("--params", type=int, default=25_000_000)
    ap.add_argument("--pad", type=int, default=0, help="extra elements per client row (row pitch)")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "sweep.json"))
    ap.add_argument("--dtype", default="f32", choices=["f32", "bf16"])
    ap.add_argument("--kernel", default="agg", choices=["agg", "fedadam", "fedyogi", "fedadagrad"],
                    help="agg: flame_agg_reduce; fedadam / fedyogi / fedadagrad: flame_fedopt_reduce_adapt (state present)")
    args = ap.parse_args()
    names = args.variants.split(",")
    if args.build:
        build_variants(names)
        return

    import torch
    from flame_amd import engine, synth
    from flame_amd import _native as N
    dev = torch.device("cuda", 0)
    n, P = args.clients, args.params
    tdt = torch.float32 if args.dtype == "f32" else torch.bfloat16
    code = N.FLAME_F32 if args.dtype == "f32" else N.FLAME_BF16
    slab = torch.empty((n, P + args.pad), dtype=tdt, device=dev)
    for i in range(n):
        engine.synth_fill_(slab[i, :P], 2, 1 + i, 0, 1e-2)
    base0 = torch.empty(P, dtype=tdt, device=dev)
    engine.synth_fill_(base0, 2, 0, 0, 1.0)
    out = torch.empty_like(base0)
    counts = synth.counts(2, n)
    rates = [int(c) / int(counts.sum()) for c in counts]
    probe = "probe" in names
    rprobe = "rprobe" in names
    names = [x for x in names if x not in ("probe", "rprobe")]
    # "<variant>:tiled" = same build, client data in the tiled [chunks][N][chunk] layout
    libs = {nm: load(nm.split(":")[0]) for nm in names}
    tiled_slab = None
    if any(nm.endswith(":tiled") for nm in names):
        T = libs[[nm for nm in names if nm.endswith(":tiled")][0]].flame_chunk_elems(code)
        S_ = -(-P // T)
        tiled_slab = torch.empty((S_, n, T), dtype=tdt, device=dev)
        engine.synth_fill_(tiled_slab.view(-1), 2, 7, 0, 1e-2)
    plans = {}
    if args.kernel != "agg":
        cur = base0.clone()
        m = torch.empty_like(base0)
        v = torch.empty_like(base0)
        engine.synth_fill_(m, 2, 9001, 0, 1e-3)
        engine.synth_fill_(v, 2, 9002, 0, 1e-3)
        v.abs_()
        cur_out = torch.empty_like(base0)
        state0 = (cur.clone(), m.clone(), v.clone())
    for nm, L in libs.items():
        if nm.endswith(":tiled"):
            T = tiled_slab.shape[2]
            # the tile must be exactly one kernel chunk, or chunk c's address runs past the slab
            if L.flame_chunk_elems(code) != T:
                raise SystemExit(f"{nm}: chunk {L.flame_chunk_elems(code)} != tile {T}; one tile size per run")
            seg = engine.Seg(P, out=out.data_ptr(), inp=base0.data_ptr(),
                             clients=[tiled_slab[0, i].data_ptr() for i in range(n)],
                             tile_stride=n * T * tiled_slab.element_size())
            if args.kernel != "agg":
                seg.cur, seg.cur_out, seg.m, seg.v = cur.data_ptr(), cur_out.data_ptr(), m.data_ptr(), v.data_ptr()
        elif args.kernel == "agg":
            seg = engine.Seg(P, out=out.data_ptr(), inp=base0.data_ptr(), clients=[slab[i].data_ptr() for i in range(n)])
        else:
            seg = engine.Seg(P, out=out.data_ptr(), inp=base0.data_ptr(), cur=cur.data_ptr(), cur_out=cur_out.data_ptr(),
                             m=m.data_ptr(), v=v.data_ptr(), clients=[slab[i].data_ptr() for i in range(n)])
        p = engine.plan(code, [seg], rates, chunk=L.flame_chunk_elems(code))
        dm = torch.from_numpy(p.meta).to(dev)
        plans[nm] = (p, dm)
    stream = torch.cuda.current_stream(dev).cuda_stream

    hyper = engine.fedopt_scalars(0.9, 0.99, 1e-2, 1e-3)

    def launch(nm):
        if nm == "probe":
            assert PL.probe_read(slab.data_ptr(), pbytes, pout.data_ptr(), 16384, 2, stream) == 0
            return
        if nm == "rprobe":    # the kernel's own per-workgroup region, 2 workgroups per CU, 6 loads per lane
            src = tiled_slab if tiled_slab is not None else slab
            assert PL.probe_read_region_persist(src.data_ptr(), pbytes, pout.data_ptr(), rregion, 6, 0, 65536,
                                                None, stream) == 0
            return
        p, dm = plans[nm]
        b = dm.data_ptr()
        if args.kernel == "agg":
            rc = libs[nm].flame_agg_reduce(code, 0, b, p.n_segs, p.n_chunks, b + p.off_clients, p.n_clients,
                                           b + p.off_r32, b + p.off_r64, stream)
        else:
            rc = libs[nm].flame_fedopt_reduce_adapt(code, {"fedadam": 0, "fedyogi": 1, "fedadagrad": 2}[args.kernel], 0, b, p.n_segs,
                                                    p.n_chunks, b + p.off_clients, p.n_clients, b + p.off_r32,
                                                    *[float(x) for x in hyper], stream)
        if rc:
            raise RuntimeError(libs[nm].flame_last_error())

    if probe:  # same-process HBM read ceiling (tools/hbm_probe.hip, best config) over the same slab
        PL = ctypes.CDLL(os.path.join(ROOT, "build", "hbm_probe.so"))
        PL.probe_read.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                  ctypes.c_void_p]
        pout = torch.zeros(4, dtype=torch.int32, device=dev)
        pbytes = slab.numel() * slab.element_size() // 4096 * 4096

        class _P:
            pass
        libs["probe"] = _P()
        plans["probe"] = None
        names = names + ["probe"]
    if rprobe:
        PL = ctypes.CDLL(os.path.join(ROOT, "build", "hbm_probe.so"))
        PL.probe_read_region_persist.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
                                                 ctypes.c_int, ctypes.c_int64, ctypes.c_int,
                                                 ctypes.POINTER(ctypes.c_int), ctypes.c_void_p]
        pout = torch.zeros(4, dtype=torch.int32, device=dev)
        src = tiled_slab if tiled_slab is not None else slab
        rregion = n * 4096 if tiled_slab is not None else 4 << 20
        pbytes = src.numel() * src.element_size() // rregion * rregion
        names = names + ["rprobe"]

    # correctness: every variant bitwise equal to the first of its layout (FedOPT: from the same
    # cur / m / v state, all four outputs compared)
    refs = {}
    for nm in names:
        if args.kernel != "agg" and nm not in ("probe", "rprobe"):
            for t, t0 in zip((cur, m, v), state0):
                t.copy_(t0)
        launch(nm)
        torch.cuda.synchronize()
        if nm in ("probe", "rprobe") or nm.startswith("nostore"):
            continue
        got = [out.clone()] if args.kernel == "agg" else [out.clone(), m.clone(), v.clone(), cur_out.clone()]
        lay = "tiled" if nm.endswith(":tiled") else "rows"
        if lay not in refs:
            refs[lay] = (nm, got)
        elif not all(torch.equal(a.view(torch.int16), b.view(torch.int16)) for a, b in zip(got, refs[lay][1])):
            raise SystemExit(f"variant {nm} differs from {refs[lay][0]}")
    print("bitwise: every variant equals the first of its layout", flush=True)
    times = {nm: [] for nm in names}
    for r in range(args.rounds):
        for nm in names:
            evs = []
            for _ in range(args.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                launch(nm)
                e1.record()
                evs.append((e0, e1))
            torch.cuda.synchronize()
            times[nm] += [a.elapsed_time(b) for a, b in evs]
        print(f"round {r} done", flush=True)
    isz = 4 if args.dtype == "f32" else 2
    nbytes = (n + 2) * P * isz if args.kernel == "agg" else (n + 8) * P * 4
    res = {}
    for nm in names:
        med, mn = statistics.median(times[nm]), min(times[nm])
        nb = pbytes if nm in ("probe", "rprobe") else nbytes
        res[nm] = {"median_ms": med, "min_ms": mn, "GBps_median": nb / med / 1e6,
                   "defs": VARIANTS.get(nm.split(":")[0], {})}
        print(f"{nm:10s} median {med:8.3f} ms  min {mn:8.3f} ms  {nb / med / 1e6:8.1f} GB/s", flush=True)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    json.dump({"clients": n, "params": P, "pad": args.pad, "results": res}, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
