#!/usr/bin/env python3
"""Per-round wall time of small rounds (flame's MNIST Net, 4 trainers, f32, HBM-resident)
through FedAvg / FedAdam / FedYogi ``do()``, synchronised; median over 50 warm rounds.

Run with FLAME_AMD_ARGMETA=0 (metadata uploaded to a device table: a blit kernel before
each launch) and without (metadata as a kernel argument) to compare the two paths.

    python tools/small_round_latency.py
"""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from examples.mnist_aggregation import MNIST_SHAPES, TrainResult  # noqa: E402


class _SortedCache(dict):
    def iterkeys(self):
        return iter(sorted(self))


def main():
    from flame_amd.optimizers import optimizer_provider
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(0)
    w0 = {k: (torch.randn(s, generator=g) * 0.05).to(dev) for k, s in MNIST_SHAPES}
    ups = [{k: v + 0.01 * (i + 1) for k, v in w0.items()} for i in range(4)]
    for sort in ["fedavg", "fedadam", "fedyogi"]:
        opt = optimizer_provider.get(sort)
        w = {k: v.clone() for k, v in w0.items()}
        times = []
        for r in range(60):
            cache = _SortedCache()
            for i, u in enumerate(ups):
                cache[f"t{i}"] = TrainResult(u, 1000 + i)
            base = {k: v.clone() for k, v in w.items()}
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            w = opt.do(base, cache, total=sum(1000 + i for i in range(4)))
            torch.cuda.synchronize()
            if r >= 10:
                times.append((time.perf_counter() - t0) * 1e3)
        print(f"argmeta={os.environ.get('FLAME_AMD_ARGMETA', '1')} {sort} 4 x MNIST f32: "
              f"median {statistics.median(times):.4f} ms  min {min(times):.4f} ms", flush=True)


if __name__ == "__main__":
    main()
