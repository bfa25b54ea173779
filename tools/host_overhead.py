#!/usr/bin/env python3
"""Host-side cost of one FedAvg.do() with 1024 slab-resident clients (cProfile top entries)."""
import cProfile
import os
import pstats
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class Cache(dict):
    def iterkeys(self):
        return iter(sorted(self))


class TR:
    def __init__(self, w, c, v=0):
        self.weights, self.count, self.version = w, c, v


def main():
    from flame_amd.optimizers import optimizer_provider
    from flame_amd.slab import UpdateSlab
    n, P = int(os.environ.get("N", 1024)), int(os.environ.get("P", 1_000_000))
    dev = torch.device("cuda", 0)
    slab = UpdateSlab({"model": torch.empty(P)}, capacity=n, device=dev)
    tmp = torch.zeros(P, device=dev)
    ws = [slab.put({"model": tmp}) for _ in range(n)]
    base = {"model": torch.zeros(P, device=dev)}
    opt = optimizer_provider.get("fedavg")

    def one():
        c = Cache()
        for i in range(n):
            c[f"{i:05d}"] = TR(ws[i], 1 + i)
        opt.do(base, c, total=n * (n + 1) // 2)

    for _ in range(3):
        one()
    torch.cuda.synchronize()
    ts = []
    for _ in range(10):
        t0 = time.perf_counter()
        one()
        ts.append(time.perf_counter() - t0)
        torch.cuda.synchronize()
    print(f"host issue per do(): median {sorted(ts)[5] * 1e3:.2f} ms (N={n})", flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(5):
        one()
    pr.disable()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("cumulative").print_stats(25)


if __name__ == "__main__":
    main()
