#!/usr/bin/env python3
"""Region pitch: a workgroup reads one contiguous region (the tiled slab's chunk row: clients x
4 KiB) and consecutive regions start `pitch` bytes apart.  Today pitch == region (16 MiB for C5,
4 MiB for C3): every concurrent workgroup's address then differs only in bits above the region
size.  Does padding the pitch (a few KiB .. 1 MiB more) spread them over the HBM channels?
~120 GB read per case; medians of 5, interleaved, one process.  python tools/region_pitch_probe.py"""
import ctypes
import os
import statistics
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "build", "hbm_probe.so")


def main():
    if not os.path.exists(SO) or "--build" in sys.argv:
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC",
                               "-o", SO, os.path.join(ROOT, "tools", "hbm_probe.hip")])
    L = ctypes.CDLL(SO)
    vp, i64 = ctypes.c_void_p, ctypes.c_int64
    L.probe_read_region.argtypes = [vp, i64, vp, i64, i64, ctypes.c_int, vp]
    nbytes = 130 << 30
    buf = torch.empty(nbytes // 4, dtype=torch.float32, device="cuda")
    buf.fill_(1.0)
    out = torch.zeros(4, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    K, M = 1 << 10, 1 << 20
    cases = []
    for region, pads in ((16 * M, (0, 4 * K, 16 * K, 64 * K, 256 * K, M + 4 * K, 2 * M)),
                         (4 * M, (0, 4 * K, 64 * K, 256 * K)),
                         (1 * M, (0, 4 * K, 64 * K))):
        for pad in pads:
            pitch = region + pad
            blocks = min((120 << 30) // region, nbytes // pitch)
            cases.append((f"region {region // M:2d} MiB pitch +{pad // K:5d} KiB", region, pitch, blocks))
    res = {c[0]: [] for c in cases}
    for _ in range(5):
        for name, region, pitch, blocks in cases:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            assert L.probe_read_region(buf.data_ptr(), blocks * pitch, out.data_ptr(), region, pitch, 16, st) == 0, name
            e1.record()
            torch.cuda.synchronize()
            res[name].append(e0.elapsed_time(e1))
    for name, region, pitch, blocks in cases:
        t = statistics.median(res[name])
        print(f"{name:40s} {t:8.3f} ms  {blocks * region / t / 1e6:8.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
