#!/usr/bin/env python3
"""cProfile of config 5's host issue per round (64 middles x 64 arrivals, slab slots, the fused
hierarchy): the middles' arrivals (batched ``FedBuff.do_arrivals`` or one ``do()`` per arrival)
and the ``hierarchy_round`` launch.  Small P -- only the host side matters here.

    python tools/hier_host_profile.py [batched|per-do] [rounds] [--sharded]
"""
import cProfile
import os
import pstats
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
    from flame_amd.optimizers import optimizer_provider
    from flame_amd.optimizer.fedbuff import hierarchy_round
    from flame_amd.slab import UpdateSlab
    mode = sys.argv[1] if len(sys.argv) > 1 else "batched"
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    sharded = "--sharded" in sys.argv       # ShardedHierarchy at world 1 (the N > 1 bench's code path)
    M, C, P, rnd = 64, 64, 1 << 20, 10
    dev = torch.device("cuda", 0)
    dt = torch.bfloat16
    if sharded:
        from flame_amd import shard
        hier = shard.ShardedHierarchy({"model": torch.empty(P, dtype=dt, device="meta")}, device=dev, middles=M)
        tmpl = hier.plan.local_template()
        src = {k: torch.zeros(v.shape, dtype=dt, device=dev) for k, v in tmpl.items()}
    else:
        tmpl = {"model": torch.empty(P, dtype=dt)}
        src = {"model": torch.zeros(P, dtype=dt, device=dev)}
    store = UpdateSlab(tmpl, capacity=M * C, device=dev)
    client_w = [store.put(src) for _ in range(M * C)]
    mid_store = UpdateSlab(tmpl, capacity=M, device=dev)
    mid_w = [mid_store.put(src) for _ in range(M)]
    gw = torch.zeros(P, dtype=dt, device=dev)
    stale = [i % 4 for i in range(M * C)]
    opts = [hier.middle_optimizer() if sharded else optimizer_provider.get("fedbuff") for _ in range(M)]

    def arrivals():
        if mode == "batched":
            return [opts[m].do_arrivals(None, [TR(client_w[i], 1, rnd - stale[i]) for i in range(m * C, (m + 1) * C)],
                                        version=rnd) for m in range(M)]
        aggs = [None] * M
        for m in range(M):
            for t in range(C):
                i = m * C + t
                c = Cache()
                c[f"{i:05d}"] = TR(client_w[i], 1, rnd - stale[i])
                aggs[m] = opts[m].do(aggs[m], c, total=1, version=rnd)
        return aggs

    def step():
        t0 = time.perf_counter()
        aggs = arrivals()
        t1 = time.perf_counter()
        rnd_fn = hier.round if sharded else hierarchy_round
        rnd_fn([(mid_w[m], aggs[m], C, rnd - (m % 2)) for m in range(M)], None, version=rnd,
               top_weights={"model": gw}, top_goal=M)
        t2 = time.perf_counter()
        return t1 - t0, t2 - t1

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    ta, tb = [], []
    for _ in range(rounds):
        a, b = step()
        ta.append(a)
        tb.append(b)
        torch.cuda.synchronize()
    ta.sort()
    tb.sort()
    print(f"{mode}{' sharded' if sharded else ''}: arrivals {ta[len(ta) // 2] * 1e3:.3f} ms, hierarchy_round issue {tb[len(tb) // 2] * 1e3:.3f} ms "
          f"(medians of {rounds})", flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(rounds):
        step()
        torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(22)


if __name__ == "__main__":
    main()
