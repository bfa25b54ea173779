#!/usr/bin/env python3
"""Mixed read/write HBM ceiling (tools/hbm_probe.hip: probe_mix_region): each workgroup
streams R x 4 KiB of reads then writes one 4 KiB block -- the reduction kernel's traffic
shape with R - 1 clients + the base per output block.  Reports GB/s of read + write bytes
for R in {2, 3, 9, 17, 33, 65, 257, 1025} over ~16 GB of reads, both store policies.

    python tools/hbm_mix_probe.py
    python tools/hbm_mix_probe.py --burst   # R = 65, writes gathered B per workgroup (probe_mix_burst)
    python tools/hbm_mix_probe.py --burst --small-r   # R = 2, 3 (FedDyn), separate or in-place writes
"""
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
        if "--build" in sys.argv:
            return
    L = ctypes.CDLL(SO)
    L.probe_mix_region.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                   ctypes.c_void_p]
    read_bytes = int(float(os.environ.get("PROBE_GB", "16")) * 1e9)
    src = torch.empty(read_bytes // 4, dtype=torch.float32, device="cuda")
    src.fill_(1.0)
    st = torch.cuda.current_stream().cuda_stream
    if "--burst" in sys.argv:
        return burst(L, src, read_bytes, st)
    for R in (2, 3, 9, 17, 33, 65, 257, 1025):
        blocks = read_bytes // (R * 4096)
        dst = torch.empty(blocks * 1024, dtype=torch.float32, device="cuda")
        for pol in (4, 0):
            ts = []
            for _ in range(6):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                assert L.probe_mix_region(src.data_ptr(), dst.data_ptr(), blocks, R, pol, st) == 0
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            t = statistics.median(ts[1:])
            rb, wb = blocks * R * 4096, blocks * 4096
            print(f"R {R:5d} : 1 write ({'sc0 sc1 nt' if pol == 4 else 'plain'}): {t:8.3f} ms  "
                  f"{(rb + wb) / t / 1e6:8.1f} GB/s (reads {rb / t / 1e6:8.1f})", flush=True)
        del dst


def burst(L, src, read_bytes, st):
    """Same R : 1 read:write ratio, writes issued B at a time at the end of a workgroup."""
    L.probe_mix_burst.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                  ctypes.c_int, ctypes.c_void_p]
    cases = [(R, B, 0) for R in (65, 257) for B in (1, 4, 16, 24, 32, 36, 1)]
    if "--small-r" in sys.argv:     # FedDyn's shapes: 2 reads (w, h) : 1 write (h'), in place or not
        cases = [(R, B, ip) for R in (2, 3) for ip in (0, 1) for B in (1, 4, 8, 16, 24, 32, 1)]
    for R, B, inplace in cases:
        if True:
            wgs = read_bytes // (R * B * 4096)
            dst = torch.empty(wgs * B * 1024, dtype=torch.float32, device="cuda")
            ts = []
            for _ in range(int(os.environ.get("PROBE_REPS", "6"))):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                rc = L.probe_mix_burst(src.data_ptr(), dst.data_ptr(), wgs, R, B, inplace, st)
                assert rc == 0, rc
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            t = statistics.median(ts[1:])
            rb, wb = wgs * B * R * 4096, wgs * B * 4096
            print(f"R {R:4d} : 1, writes{' in place' if inplace else ''} in bursts of {B:2d} ({wgs} workgroups, "
                  f"LDS {B * 4} KiB): {t:8.3f} ms  "
                  f"{(rb + wb) / t / 1e6:8.1f} GB/s", flush=True)
            del dst


if __name__ == "__main__":
    main()
