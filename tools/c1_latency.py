#!/usr/bin/env python3
"""Per-round latency of a small synchronous round (config 1: 2 trainers x MNIST Net).

Breaks one aggregator round into payload decode, cache insert (per cache placement;
the cache object lives across rounds, as the role's ``self.cache`` does), FedAvg
``do()`` issue and the wait for the GPU; medians over 25 warm rounds.  Also times
the reference's ``cloudpickle.loads`` of the same two payloads.

    python tools/c1_latency.py [--profile]
"""
import os
import statistics
import sys
import time
from copy import deepcopy

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import cloudpickle  # noqa: E402
import torch  # noqa: E402

from examples.mnist_aggregation import MNIST_SHAPES, TrainResult  # noqa: E402


class _SortedCache(dict):
    def iterkeys(self):
        return iter(sorted(self))


def main():
    from flame_amd import ingest
    from flame_amd.optimizers import optimizer_provider
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(0)
    hw = {k: torch.randn(s, generator=g) * 0.05 for k, s in MNIST_SHAPES}
    w = {k: v.to(dev) for k, v in hw.items()}
    opt = optimizer_provider.get("fedavg")
    # every round decodes FRESH payloads, as the channel delivers them: new tensors each round, so
    # the storage keys inside (the trainer's storage addresses) differ between messages
    R = 30
    rounds_pls = [[cloudpickle.dumps({"weights": {k: v + 0.01 * (i + 1) + 1e-4 * r for k, v in hw.items()},
                                      "dataset_size": 2000}) for i in range(2)] for r in range(R)]
    pls = rounds_pls[0]
    for placement in ["hbm", "slab", "host", "to_device"]:
        T = {"decode": [], "cache": [], "deepcopy": [], "do": [], "sync": [], "total": []}
        cache = _SortedCache() if placement == "to_device" else \
            ingest.DeviceUpdateCache(device=dev, placement=placement, capacity=4)
        for r in range(R):
            t0 = time.perf_counter()
            msgs = [ingest.decode(p) for p in rounds_pls[r]]
            t1 = time.perf_counter()
            for i, m in enumerate(msgs):
                if placement == "to_device":     # weights_to_model_device (common/util.py:198-208)
                    cache[f"t{i}"] = TrainResult({k: v.to(dev) for k, v in m["weights"].items()}, 2000)
                else:
                    cache[f"t{i}"] = TrainResult(m["weights"], 2000)
            t2 = time.perf_counter()
            base = deepcopy(w)           # the role's do(deepcopy(self.weights), ...) (syncfl/top_aggregator.py:161-166)
            t2b = time.perf_counter()
            opt.do(base, cache, total=4000)
            t3 = time.perf_counter()
            torch.cuda.synchronize()
            t4 = time.perf_counter()
            for k, v in zip(T, [t1 - t0, t2 - t1, t2b - t2, t3 - t2b, t4 - t3, t4 - t0]):
                T[k].append(v * 1e3)
        print(placement, {k: round(statistics.median(v[5:]), 3) for k, v in T.items()}, flush=True)
    t0 = time.perf_counter()
    for _ in range(10):
        [cloudpickle.loads(p) for p in pls]
    print(f"reference cloudpickle.loads of the 2 payloads: {(time.perf_counter() - t0) / 10 * 1e3:.3f} ms")
    if "--profile" in sys.argv:     # where a round's host time goes (slab placement)
        import cProfile
        import pstats
        cache = ingest.DeviceUpdateCache(device=dev, placement="slab", capacity=4)
        msgs = [ingest.decode(p) for p in pls]

        def rounds(n):
            for r in range(n):
                msgs = [ingest.decode(p) for p in rounds_pls[r % R]]
                for i, m in enumerate(msgs):
                    cache[f"t{i}"] = TrainResult(m["weights"], 2000)
                opt.do(deepcopy(w), cache, total=4000)
            torch.cuda.synchronize()
        rounds(5)
        pr = cProfile.Profile()
        pr.enable()
        rounds(200)
        pr.disable()
        pstats.Stats(pr).sort_stats("tottime").print_stats(30)


if __name__ == "__main__":
    main()
