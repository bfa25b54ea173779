#!/usr/bin/env python3
"""C4's FedAdam / FedYogi / FedAdaGrad spread, measured in ONE process on ONE slab.

Round 3 ran the three C4 benches one after another (14.50 / 14.86 / 14.93 ms, in that
order) on identical traffic.  Here the three optimizers take turns on the same
device-resident 1024 x 25M fp32 slab, the variant order rotating every round (Adam first,
then Yogi first, ...), so time-dependent drift (clocks, temperature) spreads evenly over
them; the kernel time is HIP events around each flame_fedopt_reduce_adapt launch.

    python tools/fedopt_spread.py --rounds 9
"""
import argparse
import json
import os
import statistics
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=1024)
    ap.add_argument("--params", type=int, default=25_000_000)
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--variants", default="fedadam,fedyogi,fedadagrad")
    a = ap.parse_args()
    from flame_amd import engine, synth
    from flame_amd.optimizers import optimizer_provider
    from flame_amd.slab import UpdateSlab
    dev = torch.device("cuda", 0)
    n, P = a.clients, a.params
    store = UpdateSlab({"model": torch.empty(P)}, capacity=n, device=dev)
    tmp = torch.empty(P, device=dev)
    ws = []
    for i in range(n):
        engine.synth_fill_(tmp, 2, 1 + i, 0, 1e-2)
        ws.append(store.put({"model": tmp}))
    engine.synth_fill_(tmp, 2, 0, 0, 1.0)
    base = tmp
    counts = synth.counts(2, n)
    total = int(counts.sum())
    names = a.variants.split(",")
    opts = {v: optimizer_provider.get(v) for v in names}
    state = {v: {"model": base.clone()} for v in names}

    def step(v):
        c = Cache()
        for i in range(n):
            c[f"{i:05d}"] = TR(ws[i], int(counts[i]))
        state[v] = opts[v].do({"model": state[v]["model"].clone()}, c, total=total)

    for v in names:       # round 1: passthrough; round 2: the first adaptive step (state zero)
        step(v)
        step(v)
    torch.cuda.synchronize()
    times = {v: [] for v in names}
    for r in range(a.rounds):
        order = names[r % len(names):] + names[:r % len(names)]
        for v in order:
            engine.kernel_events = []
            step(v)
            torch.cuda.synchronize()
            ev = [e for e in engine.kernel_events if e[0] == "flame_fedopt_reduce_adapt"]
            times[v].append(sum(e0.elapsed_time(e1) for _, e0, e1, _ in ev))
            engine.kernel_events = None
        print(f"round {r} ({','.join(order)}): " + "  ".join(f"{v} {times[v][-1]:.3f}" for v in names), flush=True)
    nbytes = 4 * P * (n + 2 + 2 + 4)
    res = {v: {"median_ms": statistics.median(t), "min_ms": min(t), "GBps": nbytes / statistics.median(t) / 1e6}
           for v, t in times.items()}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
