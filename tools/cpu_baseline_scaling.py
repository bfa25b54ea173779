#!/usr/bin/env python3
"""Why the CPU baseline scales poorly with threads.

bench.py's cpu_baseline times the reference's op sequence (oracle/torch_cpu.py: per client
``tmp = v * rate; agg += tmp``, fedavg.py:93-104), which allocates a fresh P-sized ``tmp`` per
client.  This runs that loop and the same arithmetic with ``tmp`` allocated once
(``torch.mul(v, rate, out=tmp)``) at 1..N threads over n clients x P fp32, reporting the rate
and the minor page faults each variant takes (getrusage), so the two costs can be told apart:
fresh-page faults (kernel-side, they serialise on the process's memory map) vs memory bandwidth.

    python tools/cpu_baseline_scaling.py [--clients 16] [--params 25000000] [--threads 1,2,4,8,16]
"""
import argparse
import json
import os
import resource
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=16)
    ap.add_argument("--params", type=int, default=25_000_000)
    ap.add_argument("--threads", default="1,2,4,8,16")
    a = ap.parse_args()
    from oracle import torch_cpu
    n, P = a.clients, a.params
    g = torch.Generator().manual_seed(0)
    cl = [{"w": torch.randn(P, generator=g) * 1e-2} for _ in range(n)]
    counts = list(range(1, n + 1))
    total = sum(counts)
    agg0 = torch.randn(P, generator=g)
    tmp = torch.empty(P)

    def reference(agg):
        torch_cpu.fedavg_round({"w": agg}, cl, counts, total)

    def prealloc(agg):
        for w, c in zip(cl, counts):
            torch.mul(w["w"], c / total, out=tmp)
            agg += tmp

    rows = []
    for th in [int(x) for x in a.threads.split(",")]:
        torch.set_num_threads(th)
        row = {"threads": th}
        for name, fn in (("reference", reference), ("prealloc_tmp", prealloc)):
            fn(agg0.clone())                                   # warm
            agg = agg0.clone()
            r0 = resource.getrusage(resource.RUSAGE_SELF)
            t = time.perf_counter()
            fn(agg)
            dt = time.perf_counter() - t
            r1 = resource.getrusage(resource.RUSAGE_SELF)
            row[name] = {"Gparams_per_s": n * P / dt / 1e9, "minor_faults": r1.ru_minflt - r0.ru_minflt,
                         "sys_s": r1.ru_stime - r0.ru_stime, "user_s": r1.ru_utime - r0.ru_utime, "wall_s": dt}
        rows.append(row)
        print(json.dumps(row), flush=True)
    print(json.dumps({"clients": n, "params": P, "affinity": len(os.sched_getaffinity(0)),
                      "os_cpu_count": os.cpu_count()}), flush=True)


if __name__ == "__main__":
    main()
