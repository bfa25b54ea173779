#!/usr/bin/env python3
"""Interleaved A/B sweep of compile-time variants of flame_hier_fedbuff (config 5 shard).

Each variant is a build of the PRODUCT source (flame_amd/csrc/fedagg.hip) with -DFLAME_T_*
overrides of its tunables (the defaults are the shipped kernel), loaded side by side with
ctypes; all run in ONE process on the same device-resident tiled slab (64 middles x 64
arrivals x 15.6M bf16 by default), rounds interleaved; outputs (middle weights, top
aggregate, top weights) are checked bitwise against the first variant from identical state.
A name containing "/" is a library path instead (e.g. flame_amd/libflame_amd.so).

    python tools/hier_sweep.py --build --variants base,ws    # here (hipcc cross-compiles)
    python tools/hier_sweep.py --variants base,ws --rounds 4 # on the GPU
"""
import argparse
import ctypes
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
VDIR = os.path.join(ROOT, "build", "ab", "hier")   # travels to the GPU box with the tree

# Round-2/3 sweeps of the store grouping, unroll, residency (LDS groups of 12 = 3 workgroups per
# CU), prefetch and pipelining variants are in profiles/r02_hier_*.log, r03z*_hier_sweep.log.
VARIANTS = {
    "base": {},
    "hbl12cu4": {"FLAME_T_HBL": 12, "FLAME_T_HIER_LDS_UNROLL16": 4},   # 3 workgroups per CU
}


def build_variants(names):
    from flame_amd import build as B
    os.makedirs(VDIR, exist_ok=True)
    for name in names:
        defs = [f"-D{k}={v}" for k, v in VARIANTS[name].items()]
        out = os.path.join(VDIR, f"lib_{name}.so")
        subprocess.check_call([B.hipcc(), *B.HIPCC_FLAGS, *defs, "-o", out, B.SRC])
        print("built", out, flush=True)


def load(name):
    # a name with a "/" is a library path (e.g. build/ab/lib_hnx.so, flame_amd/libflame_amd.so)
    L = ctypes.CDLL(os.path.join(ROOT, name) if "/" in name else os.path.join(VDIR, f"lib_{name}.so"))
    vp, i32, i64, u32, f32 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint, ctypes.c_float
    L.flame_hier_fedbuff.restype = ctypes.c_int
    L.flame_hier_fedbuff.argtypes = [ctypes.c_int, u32, vp, i32, i64, i32, i32, vp, vp, vp, vp, vp, vp, f32, vp]
    L.flame_last_error.restype = ctypes.c_char_p
    return L


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--variants", default="base,ws")
    ap.add_argument("--mids", type=int, default=64)
    ap.add_argument("--clients", type=int, default=64, help="arrivals per middle")
    ap.add_argument("--params", type=int, default=125_000_000 // 8)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--mid-layout", default="row", choices=["row", "tiled"],
                    help="middle weights: one tensor each, or the slots of one tiled [tiles][M][T] block")
    args = ap.parse_args()
    names = args.variants.split(",")
    if args.build:
        build_variants(sorted({n.split(":")[0] for n in names if n not in ("probe", "rprobe") and "/" not in n}))
        return

    import torch
    from flame_amd import engine
    from flame_amd import _native as N
    dev = torch.device("cuda", 0)
    M, C, P = args.mids, args.clients, args.params
    tdt = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    code = engine.dtype_code(tdt)
    T = engine.chunk_elems(code)
    tiles = -(-P // T)
    slab = torch.empty((tiles, M * C, T), dtype=tdt, device=dev)
    engine.synth_fill_(slab.view(-1), 6, 7, 0, 1e-2)
    tiled_mids = args.mid_layout == "tiled"
    mids0 = torch.empty((tiles, M, T) if tiled_mids else (M, P), dtype=tdt, device=dev)
    engine.synth_fill_(mids0.view(-1), 6, 8, 0, 1.0)
    # "<variant>:tiled" in a row-layout run: the same middles also held as one tiled block,
    # timed in the same process (layouts compared without process-to-process spread)
    tmids0 = None
    if not tiled_mids and any(nm.endswith(":tiled") for nm in names):
        tmids0 = torch.zeros((tiles, M, T), dtype=tdt, device=dev)
        tv = tmids0.permute(1, 0, 2).reshape(M, tiles * T)
        tv[:, :P].copy_(mids0)
        tmids0 = tv.view(M, tiles, T).permute(1, 0, 2).contiguous()
    gw0 = torch.empty(P, dtype=tdt, device=dev)
    engine.synth_fill_(gw0, 6, 9, 0, 1.0)
    mids, gw, top = mids0.clone(), gw0.clone(), torch.empty_like(gw0)
    tmids = tmids0.clone() if tmids0 is not None else None
    isz = slab.element_size()
    mid_ptrs = ([mids.data_ptr() + m * T * isz for m in range(M)] if tiled_mids
                else [mids[m].data_ptr() for m in range(M)])
    mts = M * T * isz if tiled_mids else 0
    seg = engine.HierSeg(P, mid_w=mid_ptrs,
                         clients=[slab.data_ptr() + i * T * isz for i in range(M * C)],
                         top_w=gw.data_ptr(), top_out=top.data_ptr(), tile_stride=M * C * T * isz,
                         mid_tile_stride=mts)
    mid_rates = [[1 / (1 + (m + t) % 4) ** 0.5 for t in range(C)] for m in range(M)]
    p = engine.plan_hier(code, [seg], mid_rates, [C] * M, [1 / (1 + m % 2) ** 0.5 for m in range(M)])
    dm = torch.from_numpy(p.meta).to(dev)
    b = dm.data_ptr()
    if tmids is not None:
        tseg = engine.HierSeg(P, mid_w=[tmids.data_ptr() + m * T * isz for m in range(M)], clients=seg.clients,
                              top_w=gw.data_ptr(), top_out=top.data_ptr(), tile_stride=seg.tile_stride,
                              mid_tile_stride=M * T * isz)
        pt = engine.plan_hier(code, [tseg], mid_rates, [C] * M, [1 / (1 + m % 2) ** 0.5 for m in range(M)])
        dmt = torch.from_numpy(pt.meta).to(dev)
        bt = dmt.data_ptr()
    stream = torch.cuda.current_stream(dev).cuda_stream
    libs = {nm: load(nm.split(":")[0]) for nm in names if nm not in ("probe", "rprobe")}
    # "<variant>:sync" = the same build in FLAME_HIER_SYNC mode (FedAvg middles + top FedAvg, same bytes)
    sseg = engine.HierSeg(P, mid_w=seg.mid_w, clients=seg.clients, top_in=gw.data_ptr(), top_out=top.data_ptr(),
                          tile_stride=seg.tile_stride, mid_tile_stride=mts)
    ps = engine.plan_hier(code, [sseg], mid_rates, [C] * M, [1 / (1 + m % 2) ** 0.5 for m in range(M)])
    dms = torch.from_numpy(ps.meta).to(dev)
    bs = dms.data_ptr()

    def launch(nm):
        if nm == "probe":
            assert PL.probe_read(slab.data_ptr(), pbytes, pout.data_ptr(), 16384, 2, stream) == 0
            return
        if nm == "rprobe":    # the kernel's own per-workgroup region at its residency and loads in flight
            assert PL.probe_read_region_persist(slab.data_ptr(), pbytes, pout.data_ptr(), M * C * T * isz, 6, 0,
                                                65536, None, stream) == 0
            return
        if nm.endswith(":sync"):
            rc = libs[nm].flame_hier_fedbuff(code, N.FLAME_HIER_TOP_ACCUM | N.FLAME_HIER_SYNC, bs + ps.offs["segs"],
                                             ps.n_segs, ps.n_chunks, M, C, bs + ps.offs["mid_w"], None,
                                             bs + ps.offs["clients"], bs + ps.offs["mid_rates"],
                                             bs + ps.offs["mid_goal"], bs + ps.offs["top_rates"], 0.0, stream)
            if rc:
                raise RuntimeError(libs[nm].flame_last_error())
            return
        pp, bb = (pt, bt) if nm.endswith(":tiled") else (p, b)
        rc = libs[nm].flame_hier_fedbuff(code, N.FLAME_HIER_TOP_APPLY, bb + pp.offs["segs"], pp.n_segs,
                                         pp.n_chunks, M, C, bb + pp.offs["mid_w"], None, bb + pp.offs["clients"],
                                         bb + pp.offs["mid_rates"], bb + pp.offs["mid_goal"],
                                         bb + pp.offs["top_rates"], float(M), stream)
        if rc:
            raise RuntimeError(libs[nm].flame_last_error())

    if "probe" in names or "rprobe" in names:
        PL = ctypes.CDLL(os.path.join(ROOT, "build", "hbm_probe.so"))
        PL.probe_read_region_persist.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
                                                 ctypes.c_int, ctypes.c_int64, ctypes.c_int,
                                                 ctypes.POINTER(ctypes.c_int), ctypes.c_void_p]
        PL.probe_read.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                  ctypes.c_void_p]
        pout = torch.zeros(4, dtype=torch.int32, device=dev)
        pbytes = slab.numel() * isz // 4096 * 4096
    refs = {}       # per mode (FedBuff / sync): every variant bitwise-equal to the first one of its mode
    for nm in names:
        if nm in ("probe", "rprobe"):
            continue
        mids.copy_(mids0)
        gw.copy_(gw0)
        if tmids is not None:
            tmids.copy_(tmids0)
        launch(nm)
        torch.cuda.synchronize()
        if nm.endswith(":tiled"):
            mlog = tmids.permute(1, 0, 2).reshape(M, tiles * T)[:, :P].clone()
        else:
            mlog = mids.clone() if not tiled_mids else mids.permute(1, 0, 2).reshape(M, tiles * T)[:, :P].clone()
        got = (mlog, gw.clone(), top.clone())
        if nm.startswith("hdiag"):
            continue
        mode = "sync" if nm.endswith(":sync") else "fedbuff"
        if mode not in refs:
            refs[mode] = (nm, got)
        elif not all(torch.equal(x.view(torch.int16), y.view(torch.int16)) for x, y in zip(got, refs[mode][1])):
            raise SystemExit(f"variant {nm} differs from {refs[mode][0]}")
    del refs
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
            times[nm] += [a.elapsed_time(b_) for a, b_ in evs]
        print(f"round {r} done", flush=True)
    nbytes = isz * P * (M * C + 2 * M + 1 + 2)
    for nm in names:
        med, mn = statistics.median(times[nm]), min(times[nm])
        nb = pbytes if nm in ("probe", "rprobe") else nbytes
        print(f"{nm:10s} median {med:8.3f} ms  min {mn:8.3f} ms  {nb / med / 1e6:8.1f} GB/s  "
              f"{VARIANTS.get(nm.split(':')[0], {})}", flush=True)


if __name__ == "__main__":
    main()
