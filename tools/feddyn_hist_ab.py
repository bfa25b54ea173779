#!/usr/bin/env python3
"""FedDyn history layouts A/B in ONE process (box-to-box spread is several %): the same
slab-resident arrivals drive three FedDyn drop-ins -- per-end histories updated in place
(``rows``), two tiled stores written alternately (``pingpong``), two tensors per end written
alternately (``pingpong_rows``) -- rounds interleaved; kernel time from HIP events; the three
results are checked bitwise every round.

    python tools/feddyn_hist_ab.py --clients 512 --params 16000000 --rounds 5
"""
import argparse
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
    ap.add_argument("--clients", type=int, default=512)
    ap.add_argument("--params", type=int, default=16_000_000)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--layouts", default="rows,pingpong,pingpong_rows")
    a = ap.parse_args()
    from flame_amd import engine
    from flame_amd.optimizers import optimizer_provider
    from flame_amd.slab import UpdateSlab
    dev = torch.device("cuda", 0)
    n, P = a.clients, a.params
    store = UpdateSlab({"model": torch.empty(P)}, capacity=n, device=dev)
    tmp = torch.empty(P, device=dev)
    ws = []
    for i in range(n):
        engine.synth_fill_(tmp, 9, 1 + i, 0, 1e-2)
        ws.append(store.put({"model": tmp}))
    engine.synth_fill_(tmp, 9, 0, 0, 1.0)
    lays = a.layouts.split(",")
    opts = {h: optimizer_provider.get("feddyn", alpha=0.01, history=h) for h in lays}
    cur = {h: {"model": tmp.clone()} for h in lays}
    ends = [f"{i:05d}" for i in range(n)]
    times = {h: [] for h in lays}
    for r in range(a.rounds + 1):
        outs = {}
        for h in (lays if r % 2 == 0 else lays[::-1]):
            opt = opts[h]
            opt.save_state("pre", active_ends=ends)
            c = Cache()
            for i, e in enumerate(ends):
                c[e] = TR(ws[i], 1)
            engine.kernel_events = []
            opt.do({"model": cur[h]["model"].clone()}, c, total=n)
            ev = engine.kernel_events
            engine.kernel_events = None
            torch.cuda.synchronize()
            cur[h] = opt.cld_model
            outs[h] = cur[h]["model"]
            if r:     # round 0 only creates the histories
                times[h].append(sum(e0.elapsed_time(e1) for nm, e0, e1, _ in ev if nm == "flame_feddyn_round"))
        first = outs[lays[0]]
        for h in lays[1:]:
            assert torch.equal(outs[h], first), f"round {r}: {h} differs from {lays[0]}"
    for h in lays:
        print(f"{h:14s} kernel median {statistics.median(times[h]):.3f} ms  ({', '.join(f'{t:.2f}' for t in times[h])})",
              flush=True)
    print("bitwise: cld_model equal across history layouts every round", flush=True)


if __name__ == "__main__":
    main()
