#!/usr/bin/env python3
"""Where config 5's hierarchy kernel spends its time, per workgroup.

A diagnostic build of the product source with stamps inserted by tools/sweep/htime.py has wave 0
of every workgroup stamp s_memrealtime (100 MHz) at: start, each middle's reduction end, each
middle's epilogue end (scale_add + delta into the top, weights into the LDS store group),
each LDS store burst's end, and the end (top scale_add).  Run on the C5 shard (64 middles x
64 arrivals x 15.6M bf16, tiled middles, FedBuff mode with the top applied) next to the
same source built without stamps (the perturbation check), then split the launch:

  streaming  -- the middles' reduction loops (arrival loads + combine)
  epilogue   -- per middle: weights load, scale_add, delta, top accumulate, LDS write
  bursts     -- the LDS-held store groups written to HBM (16 middles' weights each)
  finish     -- after the last burst: the top's scale_add (load + store of the top model)
  idle       -- workgroup slots without a workgroup (the ramp and the final partial round)

    python tools/hier_attrib.py --build          # here
    python tools/hier_attrib.py --reps 5         # on the GPU
"""
import argparse
import ctypes
import json
import os
import statistics
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
VDIR = os.path.join(ROOT, "build", "ab", "attrib")   # uploaded to the box (not in .gpurunignore)
SLOTS = 288


def build():
    from flame_amd import build as B
    sys.path.insert(0, os.path.join(ROOT, "tools", "sweep"))
    import htime
    os.makedirs(VDIR, exist_ok=True)
    stamped = htime.generate(os.path.join(VDIR, "fedagg_htime.hip"))
    for nm, src in (("base", B.SRC), ("htime", stamped)):
        subprocess.check_call([B.hipcc(), *B.HIPCC_FLAGS, "-o", os.path.join(VDIR, f"lib_{nm}.so"), src])
        print("built", nm, flush=True)


def load(nm):
    L = ctypes.CDLL(os.path.join(VDIR, f"lib_{nm}.so"))
    vp, i32, i64, u32, f32 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint, ctypes.c_float
    L.flame_hier_fedbuff.restype = ctypes.c_int
    L.flame_hier_fedbuff.argtypes = [ctypes.c_int, u32, vp, i32, i64, i32, i32, vp, vp, vp, vp, vp, vp, f32, vp]
    L.flame_last_error.restype = ctypes.c_char_p
    L.flame_hier_resident_per_cu.restype = ctypes.c_int
    L.flame_hier_resident_per_cu.argtypes = [ctypes.c_int, u32, i32]
    if hasattr(L, "flame_sweep_htime"):
        L.flame_sweep_htime.restype = ctypes.c_int
        L.flame_sweep_htime.argtypes = [vp, i32]
    return L


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--mids", type=int, default=64)
    ap.add_argument("--clients", type=int, default=64)
    ap.add_argument("--params", type=int, default=125_000_000 // 8)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    if a.build:
        build()
        return
    import torch
    from flame_amd import engine
    from flame_amd import _native as N
    dev = torch.device("cuda", 0)
    M, C, P = a.mids, a.clients, a.params
    tdt = torch.bfloat16
    code = engine.dtype_code(tdt)
    T = engine.chunk_elems(code)
    tiles = -(-P // T)
    isz = 2
    slab = torch.empty((tiles, M * C, T), dtype=tdt, device=dev)
    engine.synth_fill_(slab.view(-1), 6, 7, 0, 1e-2)
    mids = torch.empty((tiles, M, T), dtype=tdt, device=dev)
    engine.synth_fill_(mids.view(-1), 6, 8, 0, 1.0)
    gw = torch.empty(P, dtype=tdt, device=dev)
    engine.synth_fill_(gw, 6, 9, 0, 1.0)
    top = torch.empty_like(gw)
    seg = engine.HierSeg(P, mid_w=[mids.data_ptr() + m * T * isz for m in range(M)],
                         clients=[slab.data_ptr() + i * T * isz for i in range(M * C)],
                         top_w=gw.data_ptr(), top_out=top.data_ptr(), tile_stride=M * C * T * isz,
                         mid_tile_stride=M * T * isz)
    mid_rates = [[1 / (1 + (m + t) % 4) ** 0.5 for t in range(C)] for m in range(M)]
    p = engine.plan_hier(code, [seg], mid_rates, [C] * M, [1 / (1 + m % 2) ** 0.5 for m in range(M)])
    dm = torch.from_numpy(p.meta).to(dev)
    b = dm.data_ptr()
    stream = torch.cuda.current_stream(dev).cuda_stream
    plain, stamped = "base", "htime"
    libs = {"base": load(plain), "htime": load(stamped)}
    ts = torch.zeros(p.n_chunks * SLOTS, dtype=torch.int64, device=dev)
    assert libs["htime"].flame_sweep_htime(ts.data_ptr(), SLOTS) == 0
    per_cu = libs["base"].flame_hier_resident_per_cu(code, 0, M)

    def launch(nm):
        L = libs[nm]
        rc = L.flame_hier_fedbuff(code, N.FLAME_HIER_TOP_APPLY, b + p.offs["segs"], p.n_segs, p.n_chunks, M, C,
                                  b + p.offs["mid_w"], None, b + p.offs["clients"], b + p.offs["mid_rates"],
                                  b + p.offs["mid_goal"], b + p.offs["top_rates"], float(M), stream)
        if rc:
            raise RuntimeError(L.flame_last_error())

    times = {"base": [], "htime": []}
    for r in range(a.reps + 1):
        for nm in (("base", "htime") if r % 2 == 0 else ("htime", "base")):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            launch(nm)
            e1.record()
            torch.cuda.synchronize()
            if r:
                times[nm].append(e0.elapsed_time(e1))
    kms = {nm: statistics.median(t) for nm, t in times.items()}
    # the stamps of the last htime launch
    t = ts.view(p.n_chunks, SLOTS).cpu().numpy().astype(np.int64)
    nwg = p.n_chunks
    start, end = t[:, 0], t[:, 1]
    hw = t[:, 2]
    red = t[:, 3:3 + 2 * M:2]            # each middle's reduction end
    epi = t[:, 4:4 + 2 * M:2]            # each middle's epilogue end
    nb = -(-M // 16)
    burst = t[:, 3 + 2 * M:3 + 2 * M + nb]
    tick_ns = 10.0
    t0, t1 = start.min(), end.max()
    span_ms = (t1 - t0) * tick_ns / 1e6
    # per workgroup split
    prev = np.concatenate([start[:, None], epi[:, :-1]], axis=1)     # each middle's reduction starts after
    red_t = red - prev                                               # the previous epilogue (or a burst)
    for g in range(1, nb):                                           # middle 16g starts after burst g-1
        red_t[:, 16 * g] = red[:, 16 * g] - burst[:, g - 1]
    epi_t = epi - red
    burst_t = burst - epi[:, [min(16 * g + 15, M - 1) for g in range(nb)]]
    fin_t = end - burst[:, -1]
    wg_t = end - start
    tot = {k: float(v.sum()) for k, v in (("streaming", red_t), ("epilogue", epi_t), ("bursts", burst_t),
                                             ("finish", fin_t))}
    busy = float(wg_t.sum())
    slots = per_cu * 256
    idle = slots * float(t1 - t0) - busy
    # concurrency over time: how many workgroups are live
    ev = np.concatenate([np.stack([start, np.ones(nwg)], 1), np.stack([end, -np.ones(nwg)], 1)])
    ev = ev[np.argsort(ev[:, 0], kind="stable")]
    live = np.cumsum(ev[:, 1])
    full_until = ev[np.flatnonzero(live >= 0.98 * slots)[-1], 0] if np.any(live >= 0.98 * slots) else t0
    xcc = (hw >> 32) & 0xF
    res = {
        "kernel_ms_events": kms, "stamp_perturbation": kms["htime"] / kms["base"] - 1,
        "span_ms_stamps": span_ms, "workgroups": int(nwg), "slots": int(slots), "resident_per_cu": int(per_cu),
        "wg_ms": {"median": float(np.median(wg_t)) * tick_ns / 1e6, "p5": float(np.percentile(wg_t, 5)) * tick_ns / 1e6,
                  "p95": float(np.percentile(wg_t, 95)) * tick_ns / 1e6},
        "split_of_slot_time": {**{k: v / (slots * float(t1 - t0)) for k, v in tot.items()},
                               "idle": idle / (slots * float(t1 - t0))},
        "split_of_wg_time": {k: v / busy for k, v in tot.items()},
        "per_middle_us": {"streaming": float(np.median(red_t)) * tick_ns / 1e3,
                          "epilogue": float(np.median(epi_t)) * tick_ns / 1e3,
                          "burst": float(np.median(burst_t)) * tick_ns / 1e3,
                          "finish": float(np.median(fin_t)) * tick_ns / 1e3},
        "tail": {"last_full_ms": float(full_until - t0) * tick_ns / 1e6,
                 "tail_ms": float(t1 - full_until) * tick_ns / 1e6,
                 "rounds": nwg / slots},
        "xcc_workgroups": {int(x): int(np.count_nonzero(xcc == x)) for x in np.unique(xcc)},
        "wg_bytes": M * C * T * isz + 2 * M * T * isz + 2 * T * isz,
    }
    res["streaming_GBps_per_wg_while_streaming"] = (M * C * T * isz) / (float(np.median(red_t.sum(1))) * tick_ns)
    print(json.dumps(res, indent=1), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
        np.save(a.out.replace(".json", "_stamps.npy"), t[:, :3 + 2 * M + nb])


if __name__ == "__main__":
    main()
