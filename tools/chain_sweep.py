#!/usr/bin/env python3
"""Interleaved A/B of flame_fedopt_chain builds (library paths), one process: the deferred
eager FedAdam (--variant: FedYogi, FedAdaGrad) round (64 arrivals x 25M fp32 in a tiled slab) with each library swapped in as
the engine's native library, rounds alternating; chain kernel time from HIP events; base,
current, m and v checked bitwise across builds every round.
    python tools/chain_sweep.py --libs flame_amd/libflame_amd.so,build/ab/lib_chain_cu4.so
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
    def __init__(self, w, c):
        self.weights, self.count, self.version = w, c, 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", required=True)
    ap.add_argument("--arrivals", type=int, default=64)
    ap.add_argument("--params", type=int, default=25_000_000)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--dtype", default="f32", choices=["f32", "bf16", "f16"])
    ap.add_argument("--variant", default="fedadam",
                    help="fedadam | fedyogi | fedadagrad, or a comma list: every variant runs with every library, "
                         "interleaved in this one process (bitwise checked across libraries per variant)")
    a = ap.parse_args()
    variants = a.variant.split(",")
    assert all(v in ("fedadam", "fedyogi", "fedadagrad") for v in variants), variants
    from flame_amd import _native, engine, synth
    from flame_amd.optimizers import optimizer_provider
    from flame_amd.slab import UpdateSlab
    lib_names = a.libs.split(",")
    libs = {}
    for nm in lib_names:
        _native._lib, _native.LIB_PATH = None, os.path.join(ROOT, nm)
        libs[nm] = _native.lib()
    names = [(lb, v) for v in variants for lb in lib_names]
    dev = torch.device("cuda", 0)
    K, P = a.arrivals, a.params
    tdt = {"f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16}[a.dtype]
    slab = UpdateSlab({"model": torch.empty(P, dtype=tdt)}, capacity=K, device=dev)
    tmp = torch.empty(P, dtype=tdt, device=dev)
    arrivals = []
    for i in range(K):
        engine.synth_fill_(tmp, 21, 1 + i, 0, 1e-2)
        arrivals.append(slab.put({"model": tmp}))
    engine.synth_fill_(tmp, 21, 0, 0, 1.0)
    w0 = tmp.clone()
    counts = [int(c) for c in synth.counts(21, K)]
    state = {}
    for nm in names:       # each (build, variant) gets its own optimizer, past the round-1 passthrough
        _native._lib = libs[nm[0]]
        opt = optimizer_provider.get(nm[1], defer=True)
        base = {"model": w0.clone()}
        c = Cache()
        c["0"] = TR({"model": w0 * 0 + 1e-3}, 1)
        opt.do(base, c, total=1)
        state[nm] = (opt, dict(opt.current_weights))
    times = {nm: [] for nm in names}
    for r in range(a.rounds + 1):
        outs = {}
        for nm in (names if r % 2 == 0 else names[::-1]):
            _native._lib = libs[nm[0]]
            opt, weights = state[nm]
            base = {"model": weights["model"].clone()}
            total = 0
            engine.kernel_events = []
            for i in range(K):
                total += counts[i]
                c = Cache()
                c[f"{i:03d}"] = TR(arrivals[i], counts[i])
                out = opt.do(base, c, total=total)
            cur = dict(out)
            ev = engine.kernel_events
            engine.kernel_events = None
            torch.cuda.synchronize()
            state[nm] = (opt, cur)
            outs[nm] = (base["model"], cur["model"], opt.m_t["model"], opt.v_t["model"])
            if r:
                times[nm].append(sum(e0.elapsed_time(e1) for n_, e0, e1, _ in ev if n_ == "flame_fedopt_chain"))
        for nm in names:
            ref = (lib_names[0], nm[1])
            for x, y in zip(outs[nm], outs[ref]):
                assert torch.equal(x.view(torch.int16), y.view(torch.int16)), f"round {r}: {nm} differs"
        print(f"round {r} done", flush=True)
    gb = (K + 8) * P * tmp.element_size() / 1e9
    for nm in names:
        med = statistics.median(times[nm])
        print(f"{nm[1]} {a.dtype} {nm[0]:40s} chain median {med:.4f} ms  {gb / med * 1e3:.0f} GB/s  ({', '.join(f'{t:.3f}' for t in times[nm])})",
              flush=True)
    print("bitwise: base, current, m, v equal across builds every round", flush=True)


if __name__ == "__main__":
    main()
