#!/usr/bin/env python3
"""Measure the plain streaming-read ceiling (tools/hbm_probe.hip) on a 102.4 GB buffer."""
import ctypes
import json
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
    L.probe_read.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    gb = float(os.environ.get("PROBE_GB", "102.4"))
    nbytes = int(gb * 1e9) // 4096 * 4096
    buf = torch.empty(nbytes // 4, dtype=torch.float32, device="cuda")
    buf.fill_(1.0)
    out = torch.zeros(4, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    res = {}
    for blocks in (2048, 4096, 8192, 16384):
        for nt in (0, 1, 2):
            ts = []
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                assert L.probe_read(buf.data_ptr(), nbytes, out.data_ptr(), blocks, nt, st) == 0
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            t = statistics.median(ts)
            res[f"blocks{blocks}_nt{nt}"] = {"ms": t, "GBps": nbytes / t / 1e6}
            print(f"blocks {blocks:6d} nt {nt} (2: nt + 16 loads/lane): {t:8.3f} ms  {nbytes / t / 1e6:8.1f} GB/s",
                  flush=True)
    L.probe_read_region.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                    ctypes.c_int, ctypes.c_void_p]
    regions = [(1 << 20, 0), (4 << 20, 0), (16 << 20, 0), (4 << 20, 4096), (4 << 20, 1024), (4 << 20, 65536),
               (4 << 20, 256), (16 << 20, 4096), (1 << 20, 4096)]
    for region, pad in regions:
        for un in (16,):
            ts = []
            pitch = region + pad
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                assert L.probe_read_region(buf.data_ptr(), nbytes, out.data_ptr(), region, pitch, un, st) == 0
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            t = statistics.median(ts)
            rb = (nbytes // pitch) * region
            res[f"region{region >> 20}M_pad{pad}_un{un}"] = {"ms": t, "GBps": rb / t / 1e6}
            print(f"region {region >> 20:3d} MiB + pad {pad:6d} B per WG, {un} loads/lane: {t:8.3f} ms  "
                  f"{rb / t / 1e6:8.1f} GB/s", flush=True)
    L.probe_read_lds.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    for blocks in (1024, 2048, 4096):
        for nt in (0, 1):
            ts = []
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                assert L.probe_read_lds(buf.data_ptr(), nbytes, blocks, nt, st) == 0
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            t = statistics.median(ts)
            res[f"lds_blocks{blocks}_nt{nt}"] = {"ms": t, "GBps": nbytes / t / 1e6}
            print(f"LDS-DMA blocks {blocks:6d} nt {nt}: {t:8.3f} ms  {nbytes / t / 1e6:8.1f} GB/s", flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(res, open(os.path.join(ROOT, "gpurun_out", "hbm_probe.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
