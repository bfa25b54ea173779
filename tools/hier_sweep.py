#!/usr/bin/env python3
"""Interleaved A/B sweep of compile-time variants of flame_hier_fedbuff (config 5 shard).

Each variant is a separate build of flame_amd/csrc/fedagg.hip loaded side by side with
ctypes; all run in ONE process on the same device-resident tiled slab (64 middles x 64
arrivals x 15.6M bf16 by default), rounds interleaved; outputs (middle weights, top
aggregate, top weights) are checked bitwise against the first variant from identical state.

    python tools/hier_sweep.py --build            # here (hipcc cross-compiles)
    python tools/hier_sweep.py --rounds 4         # on the GPU
"""
import argparse
import ctypes
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
VDIR = os.path.join(ROOT, "build", "hvariants")

VARIANTS = {
    "base": {},
    "hcu4": {"FLAME_HCU16": 4},
    "hcu2": {"FLAME_HCU16": 2},
    "pf": {"FLAME_HPF": 1},
    "hcu4pf": {"FLAME_HCU16": 4, "FLAME_HPF": 1},
    "wpe8": {"FLAME_HWPE": 8},
    "hcu4wpe8": {"FLAME_HCU16": 4, "FLAME_HWPE": 8},
    "hcu4wpe6": {"FLAME_HCU16": 4, "FLAME_HWPE": 6},
    "hst0": {"FLAME_HST": 0},
    "hst1": {"FLAME_HST": 1},
    "hst2": {"FLAME_HST": 2},
    "hst3": {"FLAME_HST": 3},
    "hst5": {"FLAME_HST": 5},
    "hdiag1": {"FLAME_HDIAG": 1},   # diagnostic: middle weights not stored (output not checked)
    "hdiag2": {"FLAME_HDIAG": 2},   # diagnostic: middle weights neither loaded nor stored
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
    L = ctypes.CDLL(os.path.join(VDIR, f"lib_{name}.so"))
    vp, i32, i64, u32, f32 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint, ctypes.c_float
    L.flame_hier_fedbuff.restype = ctypes.c_int
    L.flame_hier_fedbuff.argtypes = [ctypes.c_int, u32, vp, i32, i64, i32, i32, vp, vp, vp, vp, vp, vp, f32, vp]
    L.flame_last_error.restype = ctypes.c_char_p
    return L


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--variants", default=",".join(VARIANTS))
    ap.add_argument("--mids", type=int, default=64)
    ap.add_argument("--clients", type=int, default=64, help="arrivals per middle")
    ap.add_argument("--params", type=int, default=125_000_000 // 8)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    args = ap.parse_args()
    names = args.variants.split(",")
    if args.build:
        build_variants(sorted({n.split(":")[0] for n in names if n != "probe"}))
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
    mids0 = torch.empty((M, P), dtype=tdt, device=dev)
    engine.synth_fill_(mids0.view(-1), 6, 8, 0, 1.0)
    gw0 = torch.empty(P, dtype=tdt, device=dev)
    engine.synth_fill_(gw0, 6, 9, 0, 1.0)
    mids, gw, top = mids0.clone(), gw0.clone(), torch.empty_like(gw0)
    isz = slab.element_size()
    seg = engine.HierSeg(P, mid_w=[mids[m].data_ptr() for m in range(M)],
                         clients=[slab.data_ptr() + i * T * isz for i in range(M * C)],
                         top_w=gw.data_ptr(), top_out=top.data_ptr(), tile_stride=M * C * T * isz)
    mid_rates = [[1 / (1 + (m + t) % 4) ** 0.5 for t in range(C)] for m in range(M)]
    p = engine.plan_hier(code, [seg], mid_rates, [C] * M, [1 / (1 + m % 2) ** 0.5 for m in range(M)])
    dm = torch.from_numpy(p.meta).to(dev)
    b = dm.data_ptr()
    stream = torch.cuda.current_stream(dev).cuda_stream
    libs = {nm: load(nm.split(":")[0]) for nm in names if nm != "probe"}
    # "<variant>:sync" = the same build in FLAME_HIER_SYNC mode (FedAvg middles + top FedAvg, same bytes)
    sseg = engine.HierSeg(P, mid_w=seg.mid_w, clients=seg.clients, top_in=gw.data_ptr(), top_out=top.data_ptr(),
                          tile_stride=seg.tile_stride)
    ps = engine.plan_hier(code, [sseg], mid_rates, [C] * M, [1 / (1 + m % 2) ** 0.5 for m in range(M)])
    dms = torch.from_numpy(ps.meta).to(dev)
    bs = dms.data_ptr()

    def launch(nm):
        if nm == "probe":
            assert PL.probe_read(slab.data_ptr(), pbytes, pout.data_ptr(), 16384, 2, stream) == 0
            return
        if nm.endswith(":sync"):
            rc = libs[nm].flame_hier_fedbuff(code, N.FLAME_HIER_TOP_ACCUM | N.FLAME_HIER_SYNC, bs + ps.offs["segs"],
                                             ps.n_segs, ps.n_chunks, M, C, bs + ps.offs["mid_w"], None,
                                             bs + ps.offs["clients"], bs + ps.offs["mid_rates"],
                                             bs + ps.offs["mid_goal"], bs + ps.offs["top_rates"], 0.0, stream)
            if rc:
                raise RuntimeError(libs[nm].flame_last_error())
            return
        rc = libs[nm].flame_hier_fedbuff(code, N.FLAME_HIER_TOP_APPLY, b + p.offs["segs"], p.n_segs, p.n_chunks,
                                         M, C, b + p.offs["mid_w"], None, b + p.offs["clients"],
                                         b + p.offs["mid_rates"], b + p.offs["mid_goal"], b + p.offs["top_rates"],
                                         float(M), stream)
        if rc:
            raise RuntimeError(libs[nm].flame_last_error())

    if "probe" in names:
        PL = ctypes.CDLL(os.path.join(ROOT, "build", "hbm_probe.so"))
        PL.probe_read.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                  ctypes.c_void_p]
        pout = torch.zeros(4, dtype=torch.int32, device=dev)
        pbytes = slab.numel() * isz // 4096 * 4096
    ref = None
    for nm in names:
        if nm == "probe":
            continue
        mids.copy_(mids0)
        gw.copy_(gw0)
        launch(nm)
        torch.cuda.synchronize()
        got = (mids.clone(), gw.clone(), top.clone())
        if nm.startswith("hdiag") or nm.endswith(":sync"):
            continue
        if ref is None:
            ref = got
        elif not all(torch.equal(x.view(torch.int16), y.view(torch.int16)) for x, y in zip(got, ref)):
            raise SystemExit(f"variant {nm} differs from {names[0]}")
    del ref
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
        nb = pbytes if nm == "probe" else nbytes
        print(f"{nm:10s} median {med:8.3f} ms  min {mn:8.3f} ms  {nb / med / 1e6:8.1f} GB/s  "
              f"{VARIANTS.get(nm.split(':')[0], {})}", flush=True)


if __name__ == "__main__":
    main()
