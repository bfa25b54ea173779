#!/usr/bin/env python3
"""Region-size question for the hierarchy kernel: read 128 GB with one workgroup
per (region, sub-row) -- tools/hbm_probe.hip read_subrow_kernel -- against contiguous regions of
the same bytes per workgroup (read_region_kernel).  Medians of 5, interleaved, one process."""
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
    L.probe_read_subrow.argtypes = [vp, i64, vp, i64, ctypes.c_int, vp]
    L.probe_read_region.argtypes = [vp, i64, vp, i64, i64, ctypes.c_int, vp]
    nbytes = (128 << 30) // (16 << 20) * (16 << 20)
    buf = torch.empty(nbytes // 4, dtype=torch.float32, device="cuda")
    buf.fill_(1.0)
    out = torch.zeros(4, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    cases = [("subrow 16MiB S=1 (C5 today)", lambda: L.probe_read_subrow(buf.data_ptr(), nbytes, out.data_ptr(), 16 << 20, 1, st)),
             ("subrow 16MiB S=2 (128-lane WG, half rows)", lambda: L.probe_read_subrow(buf.data_ptr(), nbytes, out.data_ptr(), 16 << 20, 2, st)),
             ("subrow 16MiB S=4 (64-lane WG, quarter rows)", lambda: L.probe_read_subrow(buf.data_ptr(), nbytes, out.data_ptr(), 16 << 20, 4, st)),
             ("subrow 8MiB S=1", lambda: L.probe_read_subrow(buf.data_ptr(), nbytes, out.data_ptr(), 8 << 20, 1, st)),
             ("subrow 4MiB S=1", lambda: L.probe_read_subrow(buf.data_ptr(), nbytes, out.data_ptr(), 4 << 20, 1, st)),
             ("region 16MiB (read_region_kernel)", lambda: L.probe_read_region(buf.data_ptr(), nbytes, out.data_ptr(), 16 << 20, 16 << 20, 16, st)),
             ("region 4MiB (read_region_kernel)", lambda: L.probe_read_region(buf.data_ptr(), nbytes, out.data_ptr(), 4 << 20, 4 << 20, 16, st))]
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
