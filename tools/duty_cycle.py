#!/usr/bin/env python3
"""Does the same kernel run slower when the GPU streams back to back than when launches are
spaced?  One process, one slab: FedAvg.do over K slab-resident clients (the C3 kernel at
K x P fp32; 64 x 25M = 6.4 GB, ~0.9 ms a launch) in alternating blocks of

  back-to-back -- launches queued with no host sync, the GPU never idles between them
  gap G ms     -- synchronize, sleep G ms, launch (the GPU idles G ms before each launch)

Kernel time from HIP events around each launch; median per block, blocks interleaved so a
slow drift of the box shows in both.  Written for the round-4 question why bench.py's FedBuff
top line (back-to-back steps) is 4-8 % slower than tools/fedbuff_sweep.py (isolated launches)
on the same box and the same library.

    python tools/duty_cycle.py --blocks 4 --launches 40 --gaps 1,5
"""
import argparse
import json
import os
import statistics
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=64)
    ap.add_argument("--params", type=int, default=25_000_000)
    ap.add_argument("--blocks", type=int, default=4)
    ap.add_argument("--launches", type=int, default=40)
    ap.add_argument("--gaps", default="1,5", help="idle ms before each launch in the spaced blocks")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from flame_amd import engine
    from flame_amd.optimizers import optimizer_provider
    from flame_amd.slab import UpdateSlab
    dev = torch.device("cuda", 0)
    K, P = a.clients, a.params
    store = UpdateSlab({"model": torch.empty(P)}, capacity=K, device=dev)
    tmp = torch.empty(P, device=dev)
    trs = []
    for i in range(K):
        engine.synth_fill_(tmp, 11, 1 + i, 0, 1e-2)
        trs.append((f"{i:05d}", TR(store.put({"model": tmp}), 1 + i % 7)))
    del tmp
    base = {"model": torch.zeros(P, device=dev)}
    opt = optimizer_provider.get("fedavg")
    total = sum(tr.count for _, tr in trs)
    gaps = [float(g) for g in a.gaps.split(",") if g]
    modes = ["back_to_back"] + [f"gap_{g:g}ms" for g in gaps]

    def block(mode):
        engine.kernel_events = []
        torch.cuda.synchronize()
        gap = None if mode == "back_to_back" else float(mode[4:-2]) / 1e3
        t0 = time.perf_counter()
        for _ in range(a.launches):
            if gap is not None:
                torch.cuda.synchronize()
                time.sleep(gap)
            opt.do(base, Cache(trs), total=total)     # do() pops the cache, as flame's does
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        ev = engine.kernel_events
        engine.kernel_events = None
        ks = [e0.elapsed_time(e1) for _, e0, e1, _ in ev]
        return ks, wall

    block("back_to_back")          # warm-up
    res = {m: [] for m in modes}
    busy = {m: [] for m in modes}
    for b in range(a.blocks):
        for m in (modes if b % 2 == 0 else modes[::-1]):
            ks, wall = block(m)
            res[m].append(statistics.median(ks))
            busy[m].append(sum(ks) / 1e3 / wall)
            print(f"block {b} {m:14s} median {res[m][-1]:.4f} ms  min {min(ks):.4f}  max {max(ks):.4f}  "
                  f"GPU busy {busy[m][-1]:.2f}", flush=True)
    gb = (K + 2) * P * 4 / 1e9     # K clients read, the base read and written
    summary = {m: {"median_ms": statistics.median(res[m]), "GBps": gb / statistics.median(res[m]) * 1e3,
                   "block_medians_ms": res[m], "gpu_busy": statistics.median(busy[m])} for m in modes}
    print(json.dumps({"clients": K, "params": P, "launches_per_block": a.launches, "summary": summary}), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(summary, f, indent=1)


if __name__ == "__main__":
    main()
