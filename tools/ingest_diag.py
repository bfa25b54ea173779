#!/usr/bin/env python3
"""Per-arrival cost of the shared-memory ingest into a DeviceUpdateCache, by variant (one GPU):
the same n cloudpickled 25M-fp32 updates in POSIX shm segments, received through
flame_amd.ingest.ShmReceiver and inserted with and without a shard plan, and from torch-pinned
copies for comparison.  Prints ms per arrival (decode / insert incl. its copy) per variant.

    python tools/ingest_diag.py [--clients 8] [--params 25000000]
"""
import argparse
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class TR:
    def __init__(self, w, c):
        self.weights, self.count, self.version = w, c, 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=8)
    ap.add_argument("--params", type=int, default=25_000_000)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    import cloudpickle
    from multiprocessing import shared_memory
    from flame_amd import engine, ingest, shard
    from flame_amd.ingest import DeviceUpdateCache
    from flame_amd.optimizers import optimizer_provider
    n, P = a.clients, a.params
    dev = torch.device("cuda", 0)
    tag = f"ingdiag{os.getpid()}"
    segs, sizes, pinned = [], [], []
    tmp = torch.empty(P, device=dev)
    for i in range(n):
        engine.synth_fill_(tmp, 2, 1 + i, 0, 1e-2)
        host = tmp.cpu()
        pinned.append(host.pin_memory())
        b = cloudpickle.dumps({"weights": {"model": host}, "dataset_size": 10 + i})
        s = shared_memory.SharedMemory(name=f"{tag}_t{i}-agg", create=True, size=len(b))
        s.buf[:len(b)] = b
        segs.append(s)
        sizes.append(len(b))
    try:
        rx = ingest.ShmReceiver("agg", register=True, untrack=False)
        sopt = shard.ShardedOptimizer(optimizer_provider.get("fedavg"), device=dev)
        sopt.set_layout({"model": torch.empty(P, device="meta")})
        from flame_amd import slab as S
        variants = {
            "shm -> DeviceUpdateCache(shard=plan), 3 waves, misaligned: stage": ("shm", dict(placement="slab", shard=sopt.plan)),
            "shm -> DeviceUpdateCache(shard=plan), 3 waves, misaligned: mapped": ("shm-mapped", dict(placement="slab", shard=sopt.plan)),
            "shm -> DeviceUpdateCache(slab)": ("shm", dict(placement="slab")),
            "shm -> DeviceUpdateCache(hbm)": ("shm", dict(placement="hbm")),
            "torch pinned -> DeviceUpdateCache(shard=plan)": ("pinned", dict(placement="slab", shard=sopt.plan)),
            "torch pinned -> DeviceUpdateCache(slab)": ("pinned", dict(placement="slab")),
        }
        for name, (src, kw) in variants.items():
            S.MISALIGNED_HOST = "mapped" if src == "shm-mapped" else "stage"
            src = "shm" if src == "shm-mapped" else src
            cache = DeviceUpdateCache(device=dev, capacity=n, **kw)
            dec, ins = [], []
            for r in range(a.rounds):
                for i in range(n):
                    t0 = time.perf_counter()
                    if src == "shm":
                        msg = rx.loads(f"{tag}_t{i}", sizes[i])
                        w = msg["weights"]
                        if r == 0 and i == 0:
                            v = w["model"]
                            print(f"  [{name}] decoded view: pinned={v.is_pinned()} shm={ingest.shm_lease.aliases(v) if hasattr(ingest, 'shm_lease') else '?'} "
                                  f"contiguous={v.is_contiguous()} ptr%16={v.data_ptr() % 16}", flush=True)
                    else:
                        w = {"model": pinned[i]}
                    t1 = time.perf_counter()
                    cache[f"{i:03d}"] = TR(w, 10 + i)
                    torch.cuda.synchronize()
                    t2 = time.perf_counter()
                    if r:
                        dec.append(t1 - t0)
                        ins.append(t2 - t1)
                    del w
                for i in range(n):
                    cache.pop(f"{i:03d}")
            torch.cuda.synchronize()
            gbs = P * 4 / statistics.median(ins) / 1e9
            print(f"{name:52s} decode {statistics.median(dec) * 1e3:7.3f} ms  insert {statistics.median(ins) * 1e3:7.3f} ms "
                  f"({gbs:.1f} GB/s)", flush=True)
        rx.close()
    finally:
        for s in segs:
            s.close()
            s.unlink()


if __name__ == "__main__":
    main()
