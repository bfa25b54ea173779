#!/usr/bin/env python3
"""Would smaller slab tiles help the hierarchy kernel (region size)?  Reads 128 GB
(the C5 shard's arrival bytes) as (a) today's 16 MiB per-workgroup regions in 4 KiB steps, (b)
1 KiB tiles: each wave of a 256-lane workgroup streams its own 4 MiB region (a tile row of 4,096
slots) in 1 KiB steps, (c) the same with 64-lane workgroups, (d) 4 MiB / 1 MiB regions in 4 KiB
steps for reference.  Loads in flight per lane: 16 and 6 (the hierarchy kernel's LDS-limited
figure).  Medians of 5, interleaved, one process (tools/hbm_probe.hip)."""
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
        os.makedirs(os.path.dirname(SO), exist_ok=True)
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC",
                               "-o", SO, os.path.join(ROOT, "tools", "hbm_probe.hip")])
    L = ctypes.CDLL(SO)
    vp, i64 = ctypes.c_void_p, ctypes.c_int64
    L.probe_read_region.argtypes = [vp, i64, vp, i64, i64, ctypes.c_int, vp]
    L.probe_read_wave_region.argtypes = [vp, i64, vp, i64, ctypes.c_int, ctypes.c_int, vp]
    nbytes = (128 << 30) // (16 << 20) * (16 << 20)
    buf = torch.empty(nbytes // 4, dtype=torch.float32, device="cuda")
    buf.fill_(1.0)
    out = torch.zeros(4, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    p = buf.data_ptr()
    MiB = 1 << 20
    cases = [
        ("region 16MiB 4KiB-steps un16 (C5 today)", lambda: L.probe_read_region(p, nbytes, out.data_ptr(), 16 * MiB, 16 * MiB, 16, st)),
        ("region 16MiB 4KiB-steps un8", lambda: L.probe_read_region(p, nbytes, out.data_ptr(), 16 * MiB, 16 * MiB, 8, st)),
        ("region 4MiB 4KiB-steps un16", lambda: L.probe_read_region(p, nbytes, out.data_ptr(), 4 * MiB, 4 * MiB, 16, st)),
        ("region 1MiB 4KiB-steps un16", lambda: L.probe_read_region(p, nbytes, out.data_ptr(), MiB, MiB, 16, st)),
        ("wave-region 4MiB 256-lane WG un16", lambda: L.probe_read_wave_region(p, nbytes, out.data_ptr(), 4 * MiB, 256, 16, st)),
        ("wave-region 4MiB 256-lane WG un6", lambda: L.probe_read_wave_region(p, nbytes, out.data_ptr(), 4 * MiB, 256, 6, st)),
        ("wave-region 4MiB 64-lane WG un16", lambda: L.probe_read_wave_region(p, nbytes, out.data_ptr(), 4 * MiB, 64, 16, st)),
        ("wave-region 4MiB 64-lane WG un6", lambda: L.probe_read_wave_region(p, nbytes, out.data_ptr(), 4 * MiB, 64, 6, st)),
        ("wave-region 8MiB 128-lane WG un16", lambda: L.probe_read_wave_region(p, nbytes, out.data_ptr(), 8 * MiB, 128, 16, st)),
        ("wave-region 16MiB 256-lane WG un16", lambda: L.probe_read_wave_region(p, nbytes, out.data_ptr(), 16 * MiB, 256, 16, st)),
    ]
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
        print(f"{name:44s} {t:8.3f} ms  {nbytes / t / 1e6:8.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
