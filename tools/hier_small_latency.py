#!/usr/bin/env python3
"""Per-round wall time of a small co-located synchronous hierarchy (one launch per round).

2 middles x 4 trainers over the MNIST Net shapes (config 1's model), f32: one
``sync_hierarchy_round`` per round, synchronised; median over 50 warm rounds.
Run once with FLAME_AMD_ARGMETA=0 (metadata uploaded to a device table, a blit
kernel before the reduction) and once with the default (metadata as a kernel
argument) to see what the argument path saves at this size.

    python tools/hier_small_latency.py
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
    from flame_amd.optimizer.sync_hierarchy import sync_hierarchy_round
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(0)
    top = {k: (torch.randn(s, generator=g) * 0.05).to(dev) for k, s in MNIST_SHAPES}
    mids = [{k: v.clone() for k, v in top.items()} for _ in range(2)]
    ups = [[{k: v + 0.01 * (4 * j + i + 1) for k, v in top.items()} for i in range(4)] for j in range(2)]
    times = []
    for r in range(60):
        specs = []
        for j in range(2):
            cache = _SortedCache()
            for i in range(4):
                cache[f"t{i}"] = TrainResult(ups[j][i], 1000 + i)
            specs.append((mids[j], cache, sum(1000 + i for i in range(4))))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        top, _ = sync_hierarchy_round(specs, top)
        torch.cuda.synchronize()
        if r >= 10:
            times.append((time.perf_counter() - t0) * 1e3)
    print(f"argmeta={os.environ.get('FLAME_AMD_ARGMETA', '1')} sync_hierarchy_round 2x4 MNIST f32: "
          f"median {statistics.median(times):.4f} ms  min {min(times):.4f} ms")


if __name__ == "__main__":
    main()
