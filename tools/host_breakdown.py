#!/usr/bin/env python3
"""Per-stage host cost of FedAvg.do() for N slab-resident clients (microseconds per call)."""
import os
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


def bench(label, fn, reps=200):
    fn()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    us = (time.perf_counter() - t) / reps * 1e6
    print(f"{label:28s} {us:9.1f} us", flush=True)
    return us


def main():
    from flame_amd import engine
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

    def refill():
        c = Cache()
        for i in range(n):
            c[f"{i:05d}"] = TR(ws[i], 1 + i)
        return c
    bench("cache refill", refill)
    bench("refill + _pop_entries", lambda: opt._pop_entries(refill(), total))
    entries = opt._pop_entries(refill(), total)
    keep = []
    o = base["model"]
    cs = [w["model"] for w, _ in entries]
    bench("_client_row", lambda: engine._client_row(cs, o, dev, keep))
    row, ts = engine._client_row(cs, o, dev, keep)
    seg = [engine.Seg(o.numel(), out=o.data_ptr(), inp=o.data_ptr(), clients=row, tile_stride=ts)]
    rates = [r for _, r in entries]
    bench("plan", lambda: engine.plan(0, seg, rates))
    p = engine.plan(0, seg, rates)
    bench("upload", lambda: engine._staging.upload(p.meta, dev))
    bench("reduce_ (1 key)", lambda: engine.reduce_([o], [o], [cs], rates))
    bench("accumulate", lambda: engine.accumulate(base, entries))
    bench("FedAvg.do incl. refill", lambda: opt.do(base, refill(), total=total))
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
