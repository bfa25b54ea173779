#!/usr/bin/env python3
"""Benchmark: device-resident FedAvg aggregation throughput on MI355X.

Metric (BASELINE.json): aggregated params/sec (device-resident) = N_clients * P / t,
summed over ranks.  Default workload = config 3: FedAvg of 1024 synthetic clients x
25,000,000-param fp32 updates, resident in HBM before timing.  A step is one
``FedAvg.do(base, cache, total=...)`` through flame's optimizer API (cache refill
+ client-order drain + segment table + one flame_agg_reduce launch).

Multi-GPU (torchrun, one process per GPU, RCCL): the parameter vector is sharded
-- each rank owns a 25M-param slice of a (25M x world)-param model and reduces all
1024 clients over it (weak scaling: per-GPU work fixed), then an RCCL all-gather
over xGMI reassembles the global model on every rank inside the timed step.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload fedavg|fedadam|fedyogi]
"""
import argparse
import json
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md §Chip-level parameters)


class Cache(dict):
    """diskcache.Cache surface used by the optimizers: iterkeys() in key order + pop()."""

    def iterkeys(self):
        return iter(sorted(self))


class TR:
    def __init__(self, weights, count, version=0):
        self.weights, self.count, self.version = weights, count, version


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="fedavg", choices=["fedavg", "fedadam", "fedyogi", "fedadagrad"])
    ap.add_argument("--clients", type=int, default=1024)
    ap.add_argument("--params", type=int, default=25_000_000, help="params per GPU shard")
    ap.add_argument("--seed", type=int, default=2)
    ap.add_argument("--cpu-clients", type=int, default=128, help="cpu_baseline sample size (0: skip)")
    ap.add_argument("--cpu-rounds", type=int, default=3)
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="PMC-derived HBM bytes per launch (written by tools/pmc_traffic.py)")
    return ap.parse_args()


def setup_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return world, rank, local


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def cpu_baseline(slab, base0, counts, total, n_cpu, rounds):
    """The reference's op sequence (oracle/torch_cpu.py) on host cores, bounded sample."""
    from oracle import torch_cpu
    n_cpu = min(n_cpu, slab.shape[0])
    ups = [{"model": slab[i].cpu()} for i in range(n_cpu)]
    agg = {"model": base0.cpu()}
    cts = [int(c) for c in counts[:n_cpu]]
    tot = sum(cts)
    torch_cpu.fedavg_round(agg, ups[:2], cts[:2], tot)  # warm-up
    ts = []
    for _ in range(rounds):
        t0 = time.perf_counter()
        torch_cpu.fedavg_round(agg, ups, cts, tot)
        ts.append(time.perf_counter() - t0)
    t = statistics.median(ts)
    P = slab.shape[1]
    try:
        model = [ln.split(":", 1)[1].strip() for ln in open("/proc/cpuinfo") if ln.startswith("model name")][0]
    except Exception:  # noqa: BLE001
        model = "unknown"
    return {
        "value": n_cpu * P / t, "unit": "client-params/s", "cores": torch.get_num_threads(), "kind": "port",
        "sample": f"reference FedAvg op sequence (fedavg.py:84-104, torch CPU, oracle/torch_cpu.py) over "
                  f"{n_cpu} of the same synthetic clients x {P} fp32 params, median of {rounds} rounds "
                  f"({t:.3f} s/round), {torch.get_num_threads()} threads on {model}; diskcache I/O excluded",
    }


def main():
    args = parse()
    world, rank, local = setup_dist(args)
    dev = torch.device("cuda", local)
    from flame_amd import _native, engine, synth
    from flame_amd.optimizers import optimizer_provider
    _native.lib()

    n, P = args.clients, args.params
    # ---- synthetic, device-resident inputs (counter generator; rank-specific streams)
    slab = torch.empty((n, P), dtype=torch.float32, device=dev)
    for i in range(n):
        engine.synth_fill_(slab[i], args.seed, 1 + i + rank * 100_000, 0, 1e-2)
    base = torch.empty(P, dtype=torch.float32, device=dev)
    engine.synth_fill_(base, args.seed, rank * 100_000, 0, 1.0)
    base0 = base.clone() if (rank == 0 and world == 1 and args.cpu_clients > 0) else None
    counts = synth.counts(args.seed, n)
    total = int(counts.sum())
    keys = [f"{i:05d}" for i in range(n)]
    gathered = torch.empty(P * world, dtype=torch.float32, device=dev) if world > 1 else None
    torch.cuda.synchronize()

    opt = optimizer_provider.get(args.workload)
    weights = {"model": base}

    def step():
        nonlocal weights
        cache = Cache()
        for i, k in enumerate(keys):
            cache[k] = TR({"model": slab[i]}, int(counts[i]))
        if args.workload == "fedavg":
            out = opt.do(weights, cache, total=total, num_trainers=n)
        else:  # FedOPT caller convention: do(deepcopy(weights)) -> weights
            out = opt.do({"model": weights["model"].clone()}, cache, total=total, num_trainers=n)
            weights = out
        if world > 1:
            import torch.distributed as dist
            dist.all_gather_into_tensor(gathered, out["model"])
        return out

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    engine.kernel_events = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    events = engine.kernel_events
    engine.kernel_events = None
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # dominant kernel: average duration over the timed region (HIP events on the launch stream)
    name = "flame_fedopt_reduce_adapt" if args.workload != "fedavg" else "flame_agg_reduce"
    ks = [(e0.elapsed_time(e1) / 1e3, nb) for (nm, e0, e1, nb) in events if nm == name]
    k_avg = sum(t for t, _ in ks) / len(ks)
    k_bytes = ks[0][1]
    achieved = k_bytes / k_avg / 1e9

    if rank == 0:
        traffic = None
        try:
            tr = json.load(open(args.traffic))
            if tr.get("kernel") == name and tr.get("clients") == n and tr.get("params") == P:
                traffic = tr["hbm_bytes_per_launch"]
        except Exception:  # noqa: BLE001
            pass
        cpu = None
        if world == 1 and args.cpu_clients > 0 and args.workload == "fedavg":
            cpu = cpu_baseline(slab, base0, counts, total, args.cpu_clients, args.cpu_rounds)
        value = n * P * world / (elapsed / args.steps)
        line = {
            "metric": "aggregated params/sec (device-resident), 1024-client FedAvg @1/2/4/8 GPU",
            "value": value,
            "unit": "client-params/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (counter-based generator, flame_amd/synth.py), resident in HBM",
            "config": {
                "workload": f"{args.workload}: {n} clients x {P} fp32 params per GPU"
                            + (f" (model {P * world} params, parameter-sharded, RCCL all-gather)" if world > 1 else ""),
                "clients": n, "params_per_gpu": P, "global_params": P * world,
                "parallelism": f"param-shard{world}" if world > 1 else "single",
            },
            "roofline": {
                "bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": achieved / PEAK_HBM_GBS, "traffic": traffic,
                "kernel": name, "kernel_ms": k_avg * 1e3, "algorithmic_bytes": k_bytes,
            },
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
