#!/usr/bin/env python3
"""Interleaved A/B of compile-time variants of flame_feddyn_round through the FedDyn drop-in,
in ONE process: each variant is a build of the product source with -DFLAME_T_* overrides in
build/ab/variants (tools/kernel_sweep.py --build), swapped in as the engine's native library
round by round;
the same slab-resident arrivals drive one FedDyn instance per variant; kernel time from HIP
events; cld_model checked bitwise across variants every round.

    python tools/kernel_sweep.py --build --variants base,dyncu8   # here
    python tools/feddyn_sweep.py --variants base,dyncu8 --rounds 5 # on the GPU
"""
import argparse
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
VDIR = os.path.join(ROOT, "build", "ab", "variants")   # built by tools/kernel_sweep.py --build


class Cache(dict):
    def iterkeys(self):
        return iter(sorted(self))


class TR:
    def __init__(self, w, c, v=0):
        self.weights, self.count, self.version = w, c, v


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="base")
    ap.add_argument("--clients", type=int, default=512)
    ap.add_argument("--params", type=int, default=25_000_000)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--history", default="rows")
    ap.add_argument("--order", default="sorted", choices=["sorted", "shuffled"])
    a = ap.parse_args()
    from flame_amd import _native, engine
    from flame_amd.optimizers import optimizer_provider
    from flame_amd.slab import UpdateSlab
    names = a.variants.split(",")
    libs = {}
    for nm in names:
        _native._lib, _native.LIB_PATH = None, os.path.join(VDIR, f"lib_{nm}.so")
        libs[nm] = _native.lib()
    dev = torch.device("cuda", 0)
    n, P = a.clients, a.params
    store = UpdateSlab({"model": torch.empty(P)}, capacity=n, device=dev)
    tmp = torch.empty(P, device=dev)
    ws = []
    for i in range(n):
        engine.synth_fill_(tmp, 9, 1 + i, 0, 1e-2)
        ws.append(store.put({"model": tmp}))
    engine.synth_fill_(tmp, 9, 0, 0, 1.0)
    opts = {nm: optimizer_provider.get("feddyn", alpha=0.01, history=a.history) for nm in names}
    cur = {nm: {"model": tmp.clone()} for nm in names}
    del tmp
    ends = [f"{i:05d}" for i in range(n)]
    active = list(ends)
    if a.order == "shuffled":
        g = torch.Generator().manual_seed(5)
        active = [ends[i] for i in torch.randperm(n, generator=g).tolist()]
    times = {nm: [] for nm in names}
    for r in range(a.rounds + 1):
        outs = {}
        for nm in (names if r % 2 == 0 else names[::-1]):
            _native._lib = libs[nm]
            opt = opts[nm]
            opt.save_state("pre", active_ends=active)
            c = Cache()
            for i, e in enumerate(ends):
                c[e] = TR(ws[i], 1)
            engine.kernel_events = []
            opt.do({"model": cur[nm]["model"].clone()}, c, total=n)
            ev = engine.kernel_events
            engine.kernel_events = None
            torch.cuda.synchronize()
            cur[nm] = opt.cld_model
            outs[nm] = cur[nm]["model"]
            if r:     # round 0 only creates the histories
                times[nm].append(sum(e0.elapsed_time(e1) for k, e0, e1, _ in ev if k == "flame_feddyn_round"))
        for nm in names[1:]:
            assert torch.equal(outs[nm], outs[names[0]]), f"round {r}: {nm} differs from {names[0]}"
        print(f"round {r} done", flush=True)
    gb = 3 * n * P * 4 / 1e9 + 3 * P * 4 / 1e9
    for nm in names:
        med = statistics.median(times[nm])
        print(f"{nm:12s} kernel median {med:.3f} ms  {gb / med * 1e3:.0f} GB/s  ({', '.join(f'{t:.2f}' for t in times[nm])})",
              flush=True)
    print("bitwise: cld_model equal across variants every round", flush=True)


if __name__ == "__main__":
    main()
