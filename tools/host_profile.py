#!/usr/bin/env python3
"""cProfile of the host side of FedAvg.do() on N slab-resident clients (config 2 shape):
which Python / torch calls make up the per-call issue time.

    N=256 P=1000000 python tools/host_profile.py
"""
import cProfile
import os
import pstats
import sys

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
    n, P = int(os.environ.get("N", 256)), int(os.environ.get("P", 1_000_000))
    dev = torch.device("cuda", 0)
    slab = UpdateSlab({"model": torch.empty(P)}, capacity=n, device=dev)
    tmp = torch.zeros(P, device=dev)
    ws = [slab.put({"model": tmp}) for _ in range(n)]
    base = {"model": torch.zeros(P, device=dev)}
    opt = optimizer_provider.get("fedavg")
    total = n * (n + 1) // 2
    keys = [f"{i:05d}" for i in range(n)]

    def step():
        c = Cache()
        for i in range(n):
            c[keys[i]] = TR(ws[i], 1 + i)
        opt.do(base, c, total=total)

    for _ in range(20):
        step()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(200):
        step()
    pr.disable()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
