#!/usr/bin/env python3
"""Host cost of the keys the fused FedOPT kernel does not take: a ResNet-50-like model's 53
BatchNorm ``num_batches_tracked`` (int64, 0-dim) keys beside one fp32 key, whole FedAdam
``do()`` rounds through the drop-in -- their adaptive step as ONE flame_elementwise_segments
launch (the 53 share one compiled program) -- against the same drop-in with round 5's
``_adapt_generic`` (the statements as PyTorch ops on the device, restated here), rounds
alternating in one process, GPU synchronised around each ``do()``.

    python tools/ew_overhead.py [--keys 53] [--rounds 20]
"""
import argparse
import copy
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def torch_ops_generic(self, keys, average, current, state_zero):
    """Round 5's FedOPT._adapt_generic: fedopt.py:106-129 as torch ops on the device."""
    out = {}
    for k in keys:
        d = average[k] - current[k]
        m = torch.zeros_like(d) if state_zero or k not in self.m_t else self.m_t[k]
        m = self.beta_1 * m + (1 - self.beta_1) * d
        v = torch.zeros_like(d) if state_zero or k not in self.v_t else self.v_t[k]
        v = self._delta_v_tensor(v, d)
        self.m_t[k], self.v_t[k] = m, v
        out[k] = current[k] + self.eta * m / (torch.sqrt(v) + self.tau)
    return out


class Cache(dict):
    def iterkeys(self):
        return iter(sorted(self))


class TR:
    def __init__(self, w, c):
        self.weights, self.count, self.version = w, c, 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--keys", type=int, default=53)
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--profile", action="store_true")
    ap.add_argument("--fp64", action="store_true", help="instead: an fp64 key's step, device time (fp64_rate)")
    a = ap.parse_args()
    from flame_amd.optimizers import optimizer_provider
    dev = torch.device("cuda", 0)
    keys = [f"bn{i}.num_batches_tracked" for i in range(a.keys)]
    opts = {"elementwise": optimizer_provider.get("fedadam"), "torch-ops": optimizer_provider.get("fedadam")}
    opts["torch-ops"]._adapt_generic = torch_ops_generic.__get__(opts["torch-ops"])
    w = {n: {"fc": torch.zeros(1000, device=dev), **{k: torch.tensor(7, device=dev) for k in keys}} for n in opts}
    times = {n: [] for n in opts}
    for r in range(a.rounds + 2):
        for n, opt in opts.items():
            cache = Cache()
            for i in range(4):
                cache[f"e{i}"] = TR({"fc": torch.full((1000,), 0.01 * i, device=dev),
                                      **{k: torch.tensor(7 + r + i, device=dev) for k in keys}}, 1 + i)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            w[n] = opt.do(copy.deepcopy(w[n]), cache, total=10)
            torch.cuda.synchronize()
            if r >= 2:                 # round 1 is the passthrough, round 2 compiles the program
                times[n].append(time.perf_counter() - t0)
    if a.profile:                      # where the drop-in's host time goes
        import cProfile
        import pstats
        opt = opts["elementwise"]
        pr = cProfile.Profile()
        for r in range(5):
            cache = Cache()
            for i in range(4):
                cache[f"e{i}"] = TR({"fc": torch.full((1000,), 0.01 * i, device=dev),
                                      **{k: torch.tensor(9 + r + i, device=dev) for k in keys}}, 1 + i)
            base = copy.deepcopy(w["elementwise"])
            torch.cuda.synchronize()
            pr.enable()
            w["elementwise"] = opt.do(base, cache, total=10)
            torch.cuda.synchronize()
            pr.disable()
        pstats.Stats(pr).sort_stats("tottime").print_stats(18)
    same = all(torch.equal(w["elementwise"][k].cpu(), w["torch-ops"][k].cpu()) for k in keys) if not a.profile else None
    med = {n: sorted(t)[len(t) // 2] * 1e3 for n, t in times.items()}
    print(f"{a.keys} int64 0-dim keys + 1 fp32 key, FedAdam do() (median of {a.rounds}, alternating): "
          f"elementwise programs {med['elementwise']:.2f} ms, round-5 torch ops {med['torch-ops']:.2f} ms; "
          f"num_batches_tracked results equal: {same}", flush=True)


if __name__ == "__main__" and "--fp64" not in sys.argv:
    main()


def fp64_rate(n=25_000_000, rounds=5):
    """Device time of one FedAdam adaptive step of an n-element fp64 key: the elementwise program
    (flame_elementwise, one launch) against the same statements as torch ops (round 5's path)."""
    from flame_amd.optimizers import optimizer_provider
    dev = torch.device("cuda", 0)
    opt = optimizer_provider.get("fedadam")
    g = torch.Generator(device=dev).manual_seed(3)
    avg = torch.randn(n, dtype=torch.float64, device=dev, generator=g)
    cur = torch.randn(n, dtype=torch.float64, device=dev, generator=g)
    opt.m_t = {"k": torch.randn(n, dtype=torch.float64, device=dev, generator=g) * 1e-2}
    opt.v_t = {"k": torch.rand(n, dtype=torch.float64, device=dev, generator=g) * 1e-2}
    m0, v0 = opt.m_t["k"].clone(), opt.v_t["k"].clone()
    res = {}
    for name, fn in (("elementwise", lambda: opt._adapt_generic(["k"], {"k": avg}, {"k": cur}, False)),
                     ("torch-ops", lambda: torch_ops_generic(opt, ["k"], {"k": avg}, {"k": cur}, False))):
        ts = []
        for r in range(rounds + 1):
            opt.m_t, opt.v_t = {"k": m0.clone()}, {"k": v0.clone()}
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            out = fn()
            e1.record()
            torch.cuda.synchronize()
            if r:
                ts.append(e0.elapsed_time(e1))
        res[name] = (sorted(ts)[len(ts) // 2], out["k"].clone())
    same = torch.equal(res["elementwise"][1], res["torch-ops"][1])
    gb = n * 8 * 7 / 1e9          # avg, cur, m, v read; m, v, out written
    print(f"fp64 FedAdam step, {n} elements: elementwise {res['elementwise'][0]:.3f} ms "
          f"({gb / res['elementwise'][0] * 1e3:.0f} GB/s of its {gb:.2f} GB), torch ops {res['torch-ops'][0]:.3f} ms; "
          f"bitwise equal: {same}", flush=True)


if __name__ == "__main__" and "--fp64" in sys.argv:
    fp64_rate()
