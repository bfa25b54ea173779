#!/usr/bin/env python3
"""Interleaved A/B sweep of compile-time variants of flame_agg_reduce (fp32).

Each variant is a separate build of tools/sweep/fedagg_sweep.hip (the kernel source with every sweep switch) (FLAME_BLOCK,
FLAME_CU, FLAME_VPT, FLAME_PIPE, FLAME_NT) loaded side by side with ctypes;
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
VDIR = os.path.join(ROOT, "build", "variants")

VARIANTS = {
    "base": {},
    "nt0": {"FLAME_NT": 0},
    "cu4": {"FLAME_CU": 4},
    "cu16": {"FLAME_CU": 16},
    "vpt2": {"FLAME_VPT": 2},
    "vpt2cu4": {"FLAME_VPT": 2, "FLAME_CU": 4},
    "pipe8": {"FLAME_PIPE": 1},
    "pipe4": {"FLAME_PIPE": 1, "FLAME_CU": 4},
    "b512": {"FLAME_BLOCK": 512},
    "b128": {"FLAME_BLOCK": 128},
    "b64": {"FLAME_BLOCK": 64},
    "optpf": {"FLAME_OPT_PREFETCH": 1},
    "c16_4": {"FLAME_CU16": 4},
    "c16_2": {"FLAME_CU16": 2},
    "c16_4v2": {"FLAME_CU16": 4, "FLAME_VPT": 2},
    "cu16b128": {"FLAME_CU": 16, "FLAME_BLOCK": 128},
    "stplain": {"FLAME_ST_NT": 0},
    "stnt": {"FLAME_ST_NT": 1},
    "nostore": {"FLAME_NOSTORE": 1},   # diagnostic: output not written (not checked)
    "stsc1": {"FLAME_ST_NT": 2},
    "stsc01": {"FLAME_ST_NT": 3},
    "stsc01nt": {"FLAME_ST_NT": 4},
    "wgc2": {"FLAME_WGC": 2},
    "wgc4": {"FLAME_WGC": 4},
    "wgc2d": {"FLAME_WGC": 2, "FLAME_DEFER_ST": 1},
    "wgc4d": {"FLAME_WGC": 4, "FLAME_DEFER_ST": 1},
    "wgc8d": {"FLAME_WGC": 8, "FLAME_DEFER_ST": 1},
    # FedDyn round kernel (bench.py --workload feddyn with FLAME_AMD_LIB=build/variants/lib_<name>.so)
    # FedOPT: several chunks per workgroup, outputs held in LDS and stored in one burst
    "optwgc1": {"FLAME_OPT_WGC": 1},      # round 1's FedOPT kernel (one chunk per workgroup)
    "optwgc2": {"FLAME_OPT_WGC": 2},
    "optwgc3": {"FLAME_OPT_WGC": 3},
    "optwgc4": {"FLAME_OPT_WGC": 4},
    "optwgc6": {"FLAME_OPT_WGC": 6},
    "optwgc8": {"FLAME_OPT_WGC": 8},
    "optwgc4cu16": {"FLAME_OPT_WGC": 4, "FLAME_OPT_CU": 16},
    "optwgc6cu16": {"FLAME_OPT_WGC": 6, "FLAME_OPT_CU": 16},
    "optwgc3cu16": {"FLAME_OPT_WGC": 3, "FLAME_OPT_CU": 16},
    "optwgc5": {"FLAME_OPT_WGC": 5},
    "optwgc7": {"FLAME_OPT_WGC": 7},
    "optwgc10": {"FLAME_OPT_WGC": 10},
    "optwgc8cu16": {"FLAME_OPT_WGC": 8, "FLAME_OPT_CU": 16},
    "optwgc8cu4": {"FLAME_OPT_WGC": 8, "FLAME_OPT_CU": 4},
    "dynxcd0": {"FLAME_DYN_XCD": 0},       # round-robin chunk order (before)
    "dyncu2": {"FLAME_DYN_CU": 2},
    # updated histories held in LDS, stored G steps at a time (tools/feddyn_sweep.py)
    "dynlds8": {"FLAME_DYN_LDS": 8},
    "dynlds16": {"FLAME_DYN_LDS": 16},
    "dynlds32": {"FLAME_DYN_LDS": 32},
    "dynlds16cu8": {"FLAME_DYN_LDS": 16, "FLAME_DYN_CU": 8},
    "dynlds24cu8": {"FLAME_DYN_LDS": 24, "FLAME_DYN_CU": 8},
    "dynlds12cu6": {"FLAME_DYN_LDS": 12, "FLAME_DYN_CU": 6},
    "dyncu8": {"FLAME_DYN_CU": 8},
    "dynst0": {"FLAME_DYN_ST": 0},
    "dynst1": {"FLAME_DYN_ST": 1},
    "dynst2": {"FLAME_DYN_ST": 2},
    # resident workgroups per CU capped by dynamic LDS (reduction + hierarchy kernels)
    "occ3": {"FLAME_OCC_LDS": 53248},
    "occ4": {"FLAME_OCC_LDS": 40960},
    "occ5": {"FLAME_OCC_LDS": 32768},
    "occ6": {"FLAME_OCC_LDS": 27136},
    "xcd": {"FLAME_XCD_SWIZZLE": 1},
    # round 3: fewer loads in flight per CU (tools/occ_probe.py: reads peak at 2 workgroups per CU
    # with 6 x 16-B loads per lane, above the full-occupancy configurations)
    "occ2cu6": {"FLAME_OCC_LDS": 65536, "FLAME_CU": 6},
    "occ2cu8": {"FLAME_OCC_LDS": 65536, "FLAME_CU": 8},
    "occ2cu4": {"FLAME_OCC_LDS": 65536, "FLAME_CU": 4},
    "occ2cu12": {"FLAME_OCC_LDS": 65536, "FLAME_CU": 12},
    "occ3cu4": {"FLAME_OCC_LDS": 53248, "FLAME_CU": 4},
    "occ3cu6": {"FLAME_OCC_LDS": 53248, "FLAME_CU": 6},
    "occ4cu4": {"FLAME_OCC_LDS": 40960, "FLAME_CU": 4},
    "occ2pipe3": {"FLAME_OCC_LDS": 65536, "FLAME_CU": 3, "FLAME_PIPE": 1},
    "occ2pipe4": {"FLAME_OCC_LDS": 65536, "FLAME_CU": 4, "FLAME_PIPE": 1},
    "occ2cu3": {"FLAME_OCC_LDS": 65536, "FLAME_CU": 3},
    "occ2cu2": {"FLAME_OCC_LDS": 65536, "FLAME_CU": 2},
    "occ2cu5": {"FLAME_OCC_LDS": 65536, "FLAME_CU": 5},
    "occ3cu3": {"FLAME_OCC_LDS": 53248, "FLAME_CU": 3},
    "occ3cu2": {"FLAME_OCC_LDS": 53248, "FLAME_CU": 2},
    "tailb": {"FLAME_TAILB": 1},
    "occ2cu4tb": {"FLAME_OCC_LDS": 65536, "FLAME_CU": 4, "FLAME_TAILB": 1},
    "occ2cu6tb": {"FLAME_OCC_LDS": 65536, "FLAME_CU": 6, "FLAME_TAILB": 1},
    "optwgc4cu6": {"FLAME_OPT_WGC": 4, "FLAME_OPT_CU": 6},
    "optwgc8cu12": {"FLAME_OPT_WGC": 8, "FLAME_OPT_CU": 12},
    "lo0": {"FLAME_LO_CU": 0},        # flame_agg_reduce before the low-occupancy path (full occupancy, unroll 8)
    "lo4": {"FLAME_LO_CU": 4},
    "lo2occ3": {"FLAME_LO_CU": 2, "FLAME_LO_LDS": 53248},
    "lo3occ3": {"FLAME_LO_CU": 3, "FLAME_LO_LDS": 53248},
    "optwgc4cu3": {"FLAME_OPT_WGC": 4, "FLAME_OPT_CU": 3},
    "optwgc4cu4": {"FLAME_OPT_WGC": 4, "FLAME_OPT_CU": 4},
    "bpk": {"FLAME_BF16_HI": 1, "FLAME_BF16_PK": 1},   # cheaper bf16 arithmetic (hier_sweep.py)
    "bpklo3": {"FLAME_BF16_HI": 1, "FLAME_BF16_PK": 1, "FLAME_LO_CU16": 3},
    "spf": {"FLAME_SPF": 1},          # next batch's client pointers prefetched behind the current loads
    "spflo4": {"FLAME_SPF": 1, "FLAME_LO_CU": 4},
    "spf2": {"FLAME_SPF": 2},
    # FedDyn (2 reads : 1 write) and mid-size reductions at lower residency (tools/feddyn_sweep.py)
    "dynocc2": {"FLAME_DYN_OCC_LDS": 65536},
    "dynocc2cu2": {"FLAME_DYN_OCC_LDS": 65536, "FLAME_DYN_CU": 2},
    "dynocc2cu3": {"FLAME_DYN_OCC_LDS": 65536, "FLAME_DYN_CU": 3},
    "dynocc3cu2": {"FLAME_DYN_OCC_LDS": 53248, "FLAME_DYN_CU": 2},
    "dynocc4cu2": {"FLAME_DYN_OCC_LDS": 40960, "FLAME_DYN_CU": 2},
    "lomin32": {"FLAME_LO_MIN_CLIENTS": 32},
    # the single-middle hierarchy launch (FedBuff's fused scale_add, tools/fedbuff_sweep.py) capped at
    # 2 / 3 workgroups per CU with fewer loads in flight (FLAME_CU: fp32 unroll of every full-residency path)
    "hocc2cu3": {"FLAME_OCC_LDS": 65536, "FLAME_CU": 3, "FLAME_HCU16": 4},
    "hocc2cu4": {"FLAME_OCC_LDS": 65536, "FLAME_CU": 4, "FLAME_HCU16": 4},
    "hocc3cu3": {"FLAME_OCC_LDS": 53248, "FLAME_CU": 3, "FLAME_HCU16": 3},         # FLAME_SPF >= 2 builds differ only by name (second version: rates too)
    "lo16_3": {"FLAME_LO_CU16": 3},
    "lo16_6": {"FLAME_LO_CU16": 6},
    "optwgc4cu2": {"FLAME_OPT_WGC": 4, "FLAME_OPT_CU": 2},
    "optwgc8cu3": {"FLAME_OPT_WGC": 8, "FLAME_OPT_CU": 3},
    "optwgc8cu4": {"FLAME_OPT_WGC": 8, "FLAME_OPT_CU": 4},
    "optwgc6cu3": {"FLAME_OPT_WGC": 6, "FLAME_OPT_CU": 3},
    "optwgc3cu3": {"FLAME_OPT_WGC": 3, "FLAME_OPT_CU": 3},
    "optwgc2cu3": {"FLAME_OPT_WGC": 2, "FLAME_OPT_CU": 3},
    # client loads as buffer loads with an explicit cache policy (sc0 1, nt 2, sc1 16; value - 1)
    "bl_none": {"FLAME_BUFLD": 1},
    "bl_nt": {"FLAME_BUFLD": 3},
    "bl_sc1nt": {"FLAME_BUFLD": 19},
    "bl_sc01nt": {"FLAME_BUFLD": 20},
    "bl_sc0nt": {"FLAME_BUFLD": 4},
}


def build_variants(names):
    from flame_amd import build as B
    os.makedirs(VDIR, exist_ok=True)
    for name in names:
        defs = [f"-D{k}={v}" for k, v in VARIANTS[name].items()]
        out = os.path.join(VDIR, f"lib_{name}.so")
        cmd = [B.hipcc(), *B.HIPCC_FLAGS, *defs, "-o", out, B.SWEEP_SRC]
        subprocess.check_call(cmd)
        print("built", out, flush=True)


def load(name):
    # a name with a "/" is a library path (e.g. build/diag/lib_prev.so)
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
    ap.add_argument("--kernel", default="agg", choices=["agg", "fedadam", "fedyogi"],
                    help="agg: flame_agg_reduce; fedadam/fedyogi: flame_fedopt_reduce_adapt (state present)")
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
            rc = libs[nm].flame_fedopt_reduce_adapt(code, {"fedadam": 0, "fedyogi": 1}[args.kernel], 0, b, p.n_segs,
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
