#!/usr/bin/env python3
"""Does a group-major update slab read faster than the per-chunk region layout?  128 GB read
with (a) one contiguous region per workgroup (read_region_kernel: today's tiled slab, region =
clients x 4 KiB: C3 4 MiB, C5 16 MiB) and (b) the same bytes group-major (read_blocked_kernel:
G groups of B-byte blocks, workgroups of one group neighbours).  Medians of 5, interleaved,
one process.  python tools/blocked_probe.py"""
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
    L.probe_read_blocked.argtypes = [vp, i64, vp, i64, ctypes.c_int, vp]
    nbytes = (128 << 30) // (16 << 20) * (16 << 20)
    buf = torch.empty(nbytes // 4, dtype=torch.float32, device="cuda")
    buf.fill_(1.0)
    out = torch.zeros(4, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    K = 1 << 10
    cases = [("region 16MiB (C5 slab today)", lambda: L.probe_read_region(buf.data_ptr(), nbytes, out.data_ptr(), 16 << 20, 16 << 20, 16, st)),
             ("region 4MiB (C3 slab today)", lambda: L.probe_read_region(buf.data_ptr(), nbytes, out.data_ptr(), 4 << 20, 4 << 20, 16, st)),
             ("region 1MiB", lambda: L.probe_read_region(buf.data_ptr(), nbytes, out.data_ptr(), 1 << 20, 1 << 20, 16, st))]
    for B, G in ((256 * K, 64), (256 * K, 16), (64 * K, 256), (64 * K, 64), (1 << 20, 16), (1 << 20, 4)):
        cases.append((f"blocked B={B // K}KiB G={G} ({B * G >> 20} MiB per WG)",
                      lambda B=B, G=G: L.probe_read_blocked(buf.data_ptr(), nbytes, out.data_ptr(), B, G, st)))
    res = {name: [] for name, _ in cases}
    for _ in range(5):
        for name, fn in cases:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            assert fn() == 0, name
            e1.record()
            torch.cuda.synchronize()
            res[name].append(e0.elapsed_time(e1))
    for name, ts in res.items():
        t = statistics.median(ts)
        print(f"{name:48s} {t:8.3f} ms  {nbytes / t / 1e6:8.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
