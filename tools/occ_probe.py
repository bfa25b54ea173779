#!/usr/bin/env python3
"""How much read concurrency does HBM want?  Reads 128 GB as 16 / 4 / 1 MiB per-workgroup regions
(4 KiB steps, one workgroup per region) with UN loads in flight per lane and dynamic LDS capping
the resident workgroups per CU (tools/hbm_probe.hip probe_read_region_persist).  Medians of 3,
interleaved, one process.  python tools/occ_probe.py [region MiB ...]"""
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
    L.probe_read_region_persist.argtypes = [vp, i64, vp, i64, ctypes.c_int, i64, ctypes.c_int,
                                            ctypes.POINTER(ctypes.c_int), vp]
    regions = [int(a) for a in sys.argv[1:] if a.isdigit()] or [16, 4, 1]
    nbytes = (128 << 30) // (16 << 20) * (16 << 20)
    buf = torch.empty(nbytes // 4, dtype=torch.float32, device="cuda")
    buf.fill_(1.0)
    out = torch.zeros(4, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    MiB = 1 << 20
    cases = []
    for per_cu in (1, 2, 3, 4, 8):
        lds = 0 if per_cu == 8 else (160 << 10) // per_cu - 1024
        for un in (2, 4, 6, 8, 12, 16):
            occ = ctypes.c_int(0)
            assert L.probe_read_region_persist(buf.data_ptr(), nbytes, out.data_ptr(), MiB, un, 1, lds,
                                               ctypes.byref(occ), st) == 0
            torch.cuda.synchronize()
            for reg in regions:
                name = f"{occ.value}/CU un{un:2d} region {reg:2d}MiB"
                cases.append((name, lambda reg=reg, un=un, lds=lds: L.probe_read_region_persist(
                    buf.data_ptr(), nbytes, out.data_ptr(), reg * MiB, un, 0, lds, None, st)))
    res = {name: [] for name, _ in cases}
    for _ in range(3):
        for name, fn in cases:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            assert fn() == 0, name
            e1.record()
            torch.cuda.synchronize()
            res[name].append(e0.elapsed_time(e1))
        print("pass done", flush=True)
    for name, ts in res.items():
        t = statistics.median(ts)
        print(f"{name:36s} {t:8.3f} ms  {nbytes / t / 1e6:8.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
