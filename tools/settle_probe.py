#!/usr/bin/env python3
"""After a large process exits, is the next one slow because of what its allocation got
(placement, fixed at allocation) or because of something running beside it for a while
(bandwidth taken, over once it ends)?  Buffer A (--gb) is allocated at t = 0 and its 2-per-CU
region read probe runs every --every seconds for --secs seconds; then buffer B of the same size
is allocated and both are probed.  A recovering over time = something beside it; A staying slow
while a late B is fast = placement."""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=16.0)
    ap.add_argument("--secs", type=float, default=90.0)
    ap.add_argument("--every", type=float, default=3.0)
    a = ap.parse_args()
    import bench
    n = int(a.gb * 1e9) // 4
    t0 = time.time()
    A = torch.ones(n, device="cuda")

    def rate(buf):
        best, res = bench.read_ceiling(buf, reps=3)
        return res.get("region_1MiB_2perCU_6ld", best)

    series = []
    while True:
        t = time.time() - t0
        r = rate(A)
        series.append((round(t, 1), round(r)))
        print(f"t={t:5.1f}s A {r:7.0f} GB/s", flush=True)
        if t >= a.secs:
            break
        time.sleep(a.every)
    B = torch.ones(n, device="cuda")
    ra, rb = rate(A), rate(B)
    print(f"late: A {ra:7.0f} GB/s  B (allocated at t={time.time() - t0:.0f}s) {rb:7.0f} GB/s", flush=True)
    print(json.dumps({"series_A": series, "late_A": ra, "late_B": rb}), flush=True)


if __name__ == "__main__":
    main()
