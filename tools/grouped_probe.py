#!/usr/bin/env python3
"""Would a grouped hierarchy slab help?  The C5 slab hands a workgroup one 16 MiB tile row (4,096
arrivals x 4 KiB); G slabs of 4,096 / G slots each hand it G rows of 16 / G MiB from G allocations
(no kernel change: same tile stride per slab).  Read 128 GB that way (probe_read_blocked_lds: block g of
workgroup w at (g * nwg + w) * B) against contiguous regions, at the hierarchy kernel's residency (2 per
CU, 6 loads per lane) and at full residency.  Medians of 5, interleaved, one process."""
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
    vp, i64, ci = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
    L.probe_read_region_persist.argtypes = [vp, i64, vp, i64, ci, i64, ci, ctypes.POINTER(ci), vp]
    L.probe_read_blocked_lds.argtypes = [vp, i64, vp, i64, ci, ci, ci, vp]
    nbytes = (128 << 30) // (16 << 20) * (16 << 20)
    buf = torch.empty(nbytes // 4, dtype=torch.float32, device="cuda")
    buf.fill_(1.0)
    out = torch.zeros(4, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    p, o, MiB = buf.data_ptr(), out.data_ptr(), 1 << 20
    cases = []
    for un, lds, tag in ((6, 65536, "2/CU un6"), (16, 0, "full un16")):
        for reg in (16, 4):
            cases.append((f"{tag} region {reg}MiB", lambda reg=reg, un=un, lds=lds:
                          L.probe_read_region_persist(p, nbytes, o, reg * MiB, un, 0, lds, None, st)))
        for B, G in ((8, 2), (4, 4), (2, 8), (1, 16)):
            cases.append((f"{tag} grouped G={G} x {B}MiB", lambda B=B, G=G, un=un, lds=lds:
                          L.probe_read_blocked_lds(p, nbytes, o, B * MiB, G, un, lds, st)))
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
        print(f"{name:40s} {t:8.3f} ms  {nbytes / t / 1e6:8.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
