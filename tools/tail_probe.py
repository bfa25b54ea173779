#!/usr/bin/env python3
"""Is the region-size loss a tail effect?  Long-lived workgroups (a 16 MiB region = 4 MiB of loads
per wave) dispatched one per region finish staggered over a whole workgroup lifetime at the end of
the launch, with the GPU partly idle; a persistent grid (one workgroup per resident slot, each
walking regions blockIdx.x, + grid, ...) starts and ends them together.  Reads 128 GB as 16 / 4 / 1
MiB regions, one-per-region vs persistent, at the hierarchy kernel's residency (64 KiB of LDS per
workgroup: 2 per CU, 6 loads in flight per lane) and at full residency (16 loads).  Medians of 5,
interleaved, one process (tools/hbm_probe.hip)."""
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
    nbytes = (128 << 30) // (16 << 20) * (16 << 20)
    buf = torch.empty(nbytes // 4, dtype=torch.float32, device="cuda")
    buf.fill_(1.0)
    out = torch.zeros(4, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    MiB = 1 << 20
    cases = []
    for un, lds in ((6, 64 << 10), (16, 0)):
        occ = ctypes.c_int(0)
        assert L.probe_read_region_persist(buf.data_ptr(), nbytes, out.data_ptr(), MiB, un, 1, lds, ctypes.byref(occ), st) == 0
        torch.cuda.synchronize()
        slots = occ.value * cus
        print(f"un{un} lds{lds >> 10}K: {occ.value} workgroups per CU x {cus} CUs = {slots} slots", flush=True)
        for reg in (16, 4, 1):
            for grid, tag in ((0, "one per region"), (slots, "persistent")):
                name = f"un{un} lds{lds >> 10}K region {reg:2d}MiB {tag}"
                cases.append((name, lambda reg=reg, grid=grid, un=un, lds=lds: L.probe_read_region_persist(
                    buf.data_ptr(), nbytes, out.data_ptr(), reg * MiB, un, grid, lds, None, st)))
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
