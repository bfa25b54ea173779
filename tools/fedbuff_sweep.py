#!/usr/bin/env python3
"""Interleaved A/B of compile-time variants for the async FedBuff aggregator's round
(asyncfl/top_aggregator.py:85-110: aggGoal arrivals, one per do(), then the fused
scale_add -- or a middle's scale_add + upload delta, --delta), in ONE process: each variant
is a build in build/ab/variants (tools/kernel_sweep.py --build), swapped in as the engine's
native library round by round; kernel time from HIP events; the model (and deltas) checked
bitwise across variants every round.

    python tools/kernel_sweep.py --build --variants base,lo_cu4     # here
    python tools/fedbuff_sweep.py --variants base,lo_cu4 --rounds 6  # on the GPU
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
    ap.add_argument("--arrivals", type=int, default=64)
    ap.add_argument("--params", type=int, default=25_000_000)
    ap.add_argument("--dtype", default="f32", choices=["f32", "bf16"])
    ap.add_argument("--delta", action="store_true", help="scale_add_agg_weights_with_delta (a middle's upload)")
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--stale", default="mod4", choices=["mod4", "synth"],
                    help="synth = bench.py's staleness draw (synth.counts(seed + 5, K) % 4)")
    ap.add_argument("--persistent-model", action="store_true",
                    help="one model tensor updated in place every round, as bench.py's step does "
                         "(default: a fresh clone of the start model per round)")
    a = ap.parse_args()
    from flame_amd import _native, engine
    from flame_amd.optimizers import optimizer_provider
    from flame_amd.slab import UpdateSlab
    names = a.variants.split(",")
    libs = {}
    for nm in names:
        # a name with a "/" is a library path (e.g. flame_amd/libflame_amd.so, build/ab/lib_base.so)
        path = os.path.join(ROOT, nm) if "/" in nm else os.path.join(VDIR, f"lib_{nm}.so")
        _native._lib, _native.LIB_PATH = None, path
        libs[nm] = _native.lib()
    dev = torch.device("cuda", 0)
    K, P = a.arrivals, a.params
    dt = torch.float32 if a.dtype == "f32" else torch.bfloat16
    store = UpdateSlab({"model": torch.empty(P, dtype=dt)}, capacity=K, device=dev)
    tmp = torch.empty(P, dtype=dt, device=dev)
    arrivals = []
    for i in range(K):
        engine.synth_fill_(tmp, 5, 1 + i, 0, 1e-2)
        arrivals.append(store.put({"model": tmp}))
    engine.synth_fill_(tmp, 5, 0, 0, 1.0)
    model0 = tmp.clone()
    del tmp
    if a.stale == "synth":
        from flame_amd import synth
        stale = [int(x) % 4 for x in synth.counts(5, K)]
    else:
        stale = [i % 4 for i in range(K)]
    persistent = {nm: {"model": model0.clone()} for nm in names} if a.persistent_model else None
    before = {nm: _native.launch_branch_counts() for nm in names} if len(names) == 1 else None
    rnd = 10
    times = {nm: [] for nm in names}
    for r in range(a.rounds + 1):
        outs = {}
        for nm in (names if r % 2 == 0 else names[::-1]):
            _native._lib = libs[nm]
            opt = optimizer_provider.get("fedbuff")
            model = persistent[nm] if persistent else {"model": model0.clone()}
            agg = None
            for i in range(K):
                c = Cache()
                c[f"{i:05d}"] = TR(arrivals[i], 1, rnd - stale[i])
                agg = opt.do(agg, c, total=1, version=rnd)
            torch.cuda.synchronize()
            engine.kernel_events = []
            if a.delta:
                _, d = opt.scale_add_agg_weights_with_delta(model, agg, K)
            else:
                opt.scale_add_agg_weights(model, agg, K)
                d = None
            ev = engine.kernel_events
            engine.kernel_events = None
            torch.cuda.synchronize()
            outs[nm] = (model["model"], d["model"] if d is not None else None)
            if r:
                times[nm].append(sum(e0.elapsed_time(e1) for _, e0, e1, _ in ev))
        for nm in names[1:]:
            for x, y in zip(outs[nm], outs[names[0]]):
                if x is not None:
                    assert torch.equal(x.view(torch.int16), y.view(torch.int16)), f"round {r}: {nm} differs"
        print(f"round {r} done", flush=True)
    isz = 4 if a.dtype == "f32" else 2
    gb = (K + 2 + (1 if a.delta else 0)) * P * isz / 1e9
    for nm in names:
        med = statistics.median(times[nm])
        print(f"{nm:10s} kernel median {med:.4f} ms  {gb / med * 1e3:.0f} GB/s  "
              f"({', '.join(f'{t:.3f}' for t in times[nm])})", flush=True)
    print("bitwise: model (and delta) equal across variants every round", flush=True)
    if before is not None:
        after = _native.launch_branch_counts()
        print("launch branches:", {k: v - before[names[0]][k] for k, v in after.items() if v != before[names[0]][k]},
              flush=True)


if __name__ == "__main__":
    main()
