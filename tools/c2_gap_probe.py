#!/usr/bin/env python3
"""Config 2 (256 x 1M fp32, slab): steady-state time per FedAvg round with and without the
bench's per-launch timing events, and with the metadata as kernel argument vs device table.
python tools/c2_gap_probe.py"""
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flame_amd import engine  # noqa: E402
from flame_amd.optimizers import optimizer_provider  # noqa: E402
from flame_amd.slab import UpdateSlab  # noqa: E402


class Cache(dict):
    def iterkeys(self):
        return iter(sorted(self))


class TR:
    def __init__(self, w, c):
        self.weights, self.count, self.version = w, c, 0


def main():
    n, P = 256, 1_000_000
    dev = torch.device("cuda", 0)
    slab = UpdateSlab({"model": torch.empty(P)}, capacity=n, device=dev)
    tmp = torch.empty(P, device=dev)
    ws = []
    for i in range(n):
        engine.synth_fill_(tmp, 1, 1 + i, 0, 0.01)
        ws.append(slab.put({"model": tmp}))
    base = {"model": torch.randn(P, device=dev)}
    opt = optimizer_provider.get("fedavg")
    total = n * (n + 1) // 2
    K = 400

    def run(events, argmeta):
        engine.ARGMETA = argmeta
        engine.kernel_events = [] if events else None
        caches = []
        for _ in range(K):
            c = Cache()
            for i in range(n):
                c[f"{i:05d}"] = TR(ws[i], 1 + i)
            caches.append(c)
        for c in caches[:20]:
            opt.do(base, c, total=total)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for c in caches[20:]:
            opt.do(base, c, total=total)
        torch.cuda.synchronize()
        engine.kernel_events = None
        engine.ARGMETA = True
        return (time.perf_counter() - t0) / (K - 20) * 1e6

    res = {}
    for _ in range(3):
        for events in (False, True):
            for argmeta in (True, False):
                res.setdefault((events, argmeta), []).append(run(events, argmeta))
    for (events, argmeta), v in res.items():
        print(f"events={'on ' if events else 'off'} argmeta={'on ' if argmeta else 'off'}: "
              f"{statistics.median(v):7.1f} us per round (runs {', '.join(f'{x:.1f}' for x in v)})", flush=True)


if __name__ == "__main__":
    main()
