#!/usr/bin/env python3
"""Does a physically contiguous allocation (hipExtMallocWithFlags(..., hipDeviceMallocContiguous))
stream HBM reads faster than the caching allocator's, in the state right after another large
process has exited (cross-process spread) and in a settled box?  Same process: the
read probes of bench.read_ceiling over a --gb buffer from each allocator, in --order.

    python tools/contig_probe.py --gb 102.4 --order contig,torch
"""
import argparse
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
HIP_DEVICE_MALLOC_CONTIGUOUS = 0x4


class _Dev:
    """A raw device allocation exposed to torch through __cuda_array_interface__."""

    def __init__(self, ptr, n):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "<f4", "data": (ptr, False), "version": 3}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=102.4)
    ap.add_argument("--order", default="contig,torch")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import bench
    torch.empty(1, device="cuda")
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    hip.hipFree.argtypes = [ctypes.c_void_p]
    n = int(a.gb * 1e9) // 4
    res = {}
    for kind in a.order.split(","):
        if kind == "contig":
            p = ctypes.c_void_p()
            rc = hip.hipExtMallocWithFlags(ctypes.byref(p), n * 4, HIP_DEVICE_MALLOC_CONTIGUOUS)
            if rc != 0:
                print(f"contig: hipExtMallocWithFlags rc={rc}", flush=True)
                res[kind] = None
                continue
            buf = torch.as_tensor(_Dev(p.value, n), device="cuda")
        else:
            buf = torch.empty(n, dtype=torch.float32, device="cuda")
        buf.fill_(1.0)
        best, probes = bench.read_ceiling(buf, reps=a.reps)
        res[kind] = {"best_GBps": best, **probes}
        print(kind, json.dumps({k: round(v) for k, v in res[kind].items()}), flush=True)
        torch.cuda.synchronize()
        del buf
        if kind == "contig":
            assert hip.hipFree(p) == 0
        else:
            torch.cuda.empty_cache()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
