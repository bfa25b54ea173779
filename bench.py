#!/usr/bin/env python3
"""Benchmark: device-resident server-side aggregation throughput on MI355X.

Metric (BASELINE.json): aggregated params/sec (device-resident) = clients x params
per step / step time, summed over ranks.  Default workload = config 3: FedAvg of
1024 synthetic clients x 25,000,000-param fp32 updates resident in HBM.  A step is
one ``FedAvg.do(base, cache, total=...)`` through flame's optimizer API (cache
refill + iterkeys/pop drain + segment-table upload + one flame_agg_reduce launch).

Multi-GPU (torchrun, one process per GPU, RCCL): the product's
flame_amd.shard.ShardedOptimizer(FedAvg) over a (25M x world)-param model -- each
rank owns 25M of its elements and holds only its slices of the 1024 client updates
(a rank-local tiled slab, as DeviceUpdateCache(shard=plan) writes it), reduces them
in three waves and all-gathers every wave in place over RCCL while the next wave is
reduced (weak scaling: per-GPU work fixed; the gathers are inside the timed step).

Other workloads (DESIGN.md numbers; the driver's bench line is the default):
  --workload fedadam|fedyogi|fedadagrad   config 4 (fused FedOPT kernel, round >= 2)
  --workload hier_fedbuff                 config 5: 4096 clients = 64 middles x 64, bf16,
                                          one GPU's 15.6M-param shard at N=1; at N>1 the
                                          product's ShardedHierarchy over a (15.6M x N)-param
                                          model with the top model all-gathered over RCCL
  --workload fedavg_eager [--eager-defer on|off]
                                          the eager top aggregator's round: one do() per
                                          arrival, batched into one launch (on) or not
  --workload fedadam_eager --dtype bf16   the eager FedOPT round on a 16-bit model (bf16 / f16:
                                          every op rounded to the dtype as torch-CPU does)
  --e2e                                   host-resident updates: H2D + kernel + D2H
"""
import argparse
import collections
import json
import os
import statistics
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

ISSUE_S = None  # host issue time of the timed steps (set by timed())
PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md §Chip-level parameters)
PCIE_SPEC_GBS = 64.0   # the host link: PCIe 5.0 x16, per direction, before protocol overhead
METRIC = "aggregated params/sec (device-resident), 1024-client FedAvg @1/2/4/8 GPU"


class Cache(dict):
    """diskcache.Cache surface the optimizers use: iterkeys() in key order + pop()."""

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
    ap.add_argument("--hier-mode", default="fused", choices=["fused", "group", "serial", "sync", "sync_serial"],
                    help="hier_fedbuff: the node's middles AND the top in one pass (fused, "
                         "flame_hier_fedbuff), co-located middles in one launch (group) or one by one; "
                         "sync / sync_serial: the synchronous FedAvg hierarchy (syncfl middles -> top) in one "
                         "FLAME_HIER_SYNC launch or as the roles' separate FedAvg.do + delta calls")
    ap.add_argument("--hier-middles", default="own", choices=["own", "fetched"],
                    help="hier_fedbuff fused: own = every middle keeps its own weights, updated in place; "
                         "fetched = the middles hold the top model they fetched this round (one shared "
                         "tensor, read-only: their updated weights only feed the upload delta and are "
                         "replaced at the next fetch, asyncfl/middle_aggregator.py:119-120,244-246)")
    ap.add_argument("--hier-mid-layout", default="tiled", choices=["tiled", "row"],
                    help="hier_fedbuff own middles (fused / sync modes): the middles' weights as the slots of "
                         "one tiled UpdateSlab (a chunk's middles are one contiguous block) or one tensor each")
    ap.add_argument("--workload", default="fedavg",
                    choices=["fedavg", "fedadam", "fedyogi", "fedadagrad", "fedbuff", "hier_fedbuff", "feddyn",
                             "scaffold", "fedavg_eager", "fedadam_eager", "fedyogi_eager", "fedadagrad_eager"])
    ap.add_argument("--dtype", default="f32", choices=["f32", "bf16", "f16"],
                    help="fed*_eager: the model's and the updates' dtype (the eager FedOPT chain ships for all "
                         "three, each op rounded to the dtype as torch-CPU does); every other workload runs its "
                         "BASELINE config's dtype")
    ap.add_argument("--eager-defer", default="on", choices=["on", "off"],
                    help="fed*_eager / --e2e-mode eager: FedAvg / FedOPT(defer=True) queues the one-arrival do() "
                         "calls and reduces them in one launch (on) or launches per arrival (off)")
    ap.add_argument("--fedbuff-fuse", default="on", choices=["on", "off"],
                    help="fedbuff: scale_add straight from the queued arrivals (on) or flush + scale_add (off)")
    ap.add_argument("--feddyn-order", default="sorted", choices=["sorted", "shuffled"],
                    help="feddyn: active_ends order (sorted = the cache order: one merged pass)")
    ap.add_argument("--feddyn-history", default="rows", choices=["pingpong", "pingpong_rows", "rows"],
                    help="feddyn: per-end histories in two tiled stores written alternately, or one "
                         "tensor per end updated in place")
    ap.add_argument("--clients", type=int, default=None, help="default 1024 (hier_fedbuff: 64 x 64)")
    ap.add_argument("--params", type=int, default=None,
                    help="params per GPU (default 25,000,000; hier_fedbuff 125M/8 = 15,625,000)")
    ap.add_argument("--seed", type=int, default=2)
    ap.add_argument("--no-overlap", action="store_true", help="N>1: do not pipeline the all-gather")
    ap.add_argument("--hier-arrivals", default="batched", choices=["batched", "per-do"],
                    help="hier_fedbuff fused: each middle's round of arrivals in ONE FedBuff.do_arrivals call "
                         "(batched) or one do() per arrival as the async middle role issues them (per-do)")
    ap.add_argument("--hier-wave-quantum", default="on", choices=["on", "off"],
                    help="sharded hierarchy: size the last wave to whole rounds of resident workgroups")
    ap.add_argument("--shard-fracs", default=None,
                    help="N>1: element fractions of the waves, e.g. 0.9,0.1 (default: flame_amd.shard's)")
    ap.add_argument("--force-shard", action="store_true",
                    help="run the N>1 code path (process group + sharded FedAvg + all-gather) even at N=1 "
                         "(rehearses the RCCL path on a one-GPU box under torchrun)")
    ap.add_argument("--layout", default="slab", choices=["slab", "row"],
                    help="slab: updates in the tiled UpdateSlab (what DeviceUpdateCache produces); "
                         "row: one contiguous tensor per client (weights_to_model_device layout)")
    ap.add_argument("--e2e", action="store_true", help="host-resident updates (end-to-end)")
    ap.add_argument("--e2e-mode", default="zerocopy",
                    choices=["zerocopy", "copy", "pageable", "wire", "wire_pinned", "wire_reference", "eager",
                             "shm", "shm_reference", "shard", "shm_shard"],
                    help="zerocopy: kernel streams pinned host memory; copy: pinned -> HBM on a copy "
                         "stream overlapped with the reduction; pageable: reference weights_to_model_device; "
                         "shm at N > 1 (or shm_shard at any N): the sharded shm ingest + gathers + egress encode")
    ap.add_argument("--e2e-egress", default="sharded", choices=["sharded", "gathered"],
                    help="N-GPU shm line: sharded = no all-gather, every rank D2Hs its ranges into one shared "
                         "payload (flame_amd.egress.ShardedEgress); gathered = in-place all-gathers, then rank 0 "
                         "encodes the whole model (MessageEncoder)")
    ap.add_argument("--e2e-placement", default="slab", choices=["slab", "hbm"],
                    help="eager mode: DeviceUpdateCache placement of the arriving updates")
    ap.add_argument("--cpu-clients", type=int, default=128, help="cpu_baseline sample size (0: skip)")
    ap.add_argument("--cpu-rounds", type=int, default=3)
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="PMC-derived HBM bytes per launch (tools/gpu_prof.sh -> tools/pmc_traffic.py)")
    return ap.parse_args()


def setup_dist(force_group=False):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU; FLAME_BENCH_BACKEND=gloo lets several ranks share one GPU to
    # rehearse the N>1 path on a single-GPU box (the driver's N>1 runs use RCCL = "nccl")
    backend = os.environ.get("FLAME_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local = local % torch.cuda.device_count()
    torch.cuda.set_device(local)
    if world > 1 or force_group:
        import torch.distributed as dist
        if "RANK" not in os.environ:      # --force-shard without torchrun: a world-1 group
            import socket
            sk = socket.socket()
            sk.bind(("127.0.0.1", 0))
            os.environ.update(RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
                              MASTER_PORT=str(sk.getsockname()[1]))
            sk.close()
        # bounded: a rank that never joins (or a hung collective, RCCL aborts on it) fails the run in
        # minutes instead of the default ten
        import datetime
        tmo = datetime.timedelta(seconds=int(os.environ.get("FLAME_BENCH_PG_TIMEOUT", "300")))
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=tmo)
        else:
            dist.init_process_group(backend, timeout=tmo)
    return world, rank, local


def process_group_info():
    """The process group the line was measured over (None without one)."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return None
    return {"backend": dist.get_backend(), "world": dist.get_world_size()}


def barrier(world):
    import torch.distributed as dist
    if world > 1 or (dist.is_available() and dist.is_initialized()):
        import torch.distributed as dist
        dist.barrier()


def host_cores():
    """The host cores this process may use, with the figures they come from (SURVEY.md
    §8(d): state the core count).  A GPU box pins a job to a CPU share: the affinity mask
    and the cgroup quota bound it; os.cpu_count() is the whole machine."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(period)))
    except Exception:  # noqa: BLE001
        pass
    use = min(aff, quota) if quota else aff
    return use, {"os_cpu_count": os.cpu_count(), "sched_getaffinity": aff, "cgroup_cpu_quota": quota,
                 "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS"), "threads_used": use, "cpu_model": _cpu_model()}


def cpu_baseline(host_row, n, P, base0, counts, n_cpu, rounds):
    """The reference's op sequence (oracle/torch_cpu.py) on host cores, bounded sample,
    with torch's intra-op pool set to the cores this process may use (host_cores)."""
    cores, env = host_cores()
    prev = torch.get_num_threads()
    torch.set_num_threads(cores)
    try:
        res = _cpu_baseline(host_row, n, P, base0, counts, n_cpu, rounds)
    finally:
        torch.set_num_threads(prev)
    res["host"] = env
    return res


def _cpu_baseline(host_row, n, P, base0, counts, n_cpu, rounds):
    from oracle import torch_cpu
    n_cpu = min(n_cpu, n)
    ups = [{"model": host_row(i)} for i in range(n_cpu)]
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
    model = _cpu_model()
    # also one thread (a smaller sample keeps it to a few seconds)
    threads = torch.get_num_threads()
    n1 = min(16, n_cpu)
    torch.set_num_threads(1)
    try:
        t1s = []
        for _ in range(rounds):
            t0 = time.perf_counter()
            torch_cpu.fedavg_round(agg, ups[:n1], cts[:n1], tot)
            t1s.append(time.perf_counter() - t0)
    finally:
        torch.set_num_threads(threads)
    t1 = statistics.median(t1s)
    return {
        "value": n_cpu * P / t, "unit": "client-params/s", "cores": threads, "kind": "port",
        "sample": f"reference FedAvg op sequence (fedavg.py:84-104, torch CPU, oracle/torch_cpu.py) over "
                  f"{n_cpu} of the same synthetic clients x {P} fp32 params, median of {rounds} rounds "
                  f"({t:.3f} s/round), {threads} threads on {model}; diskcache I/O excluded.  value = sampled "
                  f"client-params / round time: the op sequence costs the same per client, so this is the "
                  f"{n}-client rate extrapolated per-client-linearly ({n} clients would take "
                  f"{t * n / n_cpu:.1f} s)",
        "single_thread": {"value": n1 * P / t1, "cores": 1,
                          "sample": f"{n1} clients x {P}, median of {rounds} rounds ({t1:.3f} s/round)"},
    }


def _cpu_model():
    try:
        return [ln.split(":", 1)[1].strip() for ln in open("/proc/cpuinfo") if ln.startswith("model name")][0]
    except Exception:  # noqa: BLE001
        return "unknown"


def cpu_baseline_fedopt(sort, host_row, n, P, base0, counts, n_cpu, rounds):
    """FedAvg over a client sample + one adaptive step (fedopt.py:102-129), reference op
    sequence on host cores; value = sampled client-params / time of that round."""
    from oracle import torch_cpu
    n_cpu = min(n_cpu, n)
    ups = [{"model": host_row(i)} for i in range(n_cpu)]
    cts = [int(c) for c in counts[:n_cpu]]
    tot = sum(cts)
    cur = {"model": base0.cpu()}
    ts, ta = [], []
    for r in range(rounds + 1):
        agg = {"model": cur["model"].clone()}
        t0 = time.perf_counter()
        torch_cpu.fedavg_round(agg, ups, cts, tot)
        t1 = time.perf_counter()
        torch_cpu.fedopt_adapt(sort, agg, cur, {}, {}, 0.9, 0.99, 1e-2, 1e-3)
        t2 = time.perf_counter()
        if r:
            ts.append(t2 - t0)
            ta.append(t2 - t1)
    t = statistics.median(ts)
    return {
        "value": n_cpu * P / t, "unit": "client-params/s", "cores": torch.get_num_threads(), "kind": "port",
        "sample": f"reference {sort} op sequence (fedavg.py:84-104 + fedopt.py:102-129, torch CPU, "
                  f"oracle/torch_cpu.py): FedAvg over {n_cpu} of the same synthetic clients x {P} fp32 params "
                  f"+ one adaptive step, median of {rounds} ({t:.3f} s/round, of which adapt "
                  f"{statistics.median(ta):.3f} s), {torch.get_num_threads()} threads on {_cpu_model()}",
    }


def cpu_baseline_eager(sort, host_row, n, P, base0, counts, n_cpu, rounds):
    """The eager top aggregator's round (eager_syncfl/top_aggregator.py:36-90) as the reference
    runs it, on host cores: per arrival, FedAvg.do of that one arrival into the round's base with
    the running total (fedavg.py:84-104) and, for FedOPT, the adaptive step (fedopt.py:102-129)
    with m / v / current carried from arrival to arrival -- every op in the model's dtype, as
    torch-CPU rounds it.  A bounded sample: the round's first ``n_cpu`` arrivals, one untimed
    round first (it allocates m / v), the median of ``rounds``; value = arrivals x P / time."""
    from oracle import torch_cpu
    cores, env = host_cores()
    prev = torch.get_num_threads()
    torch.set_num_threads(cores)
    fedopt = sort != "fedavg"
    n_cpu = max(1, min(n_cpu, n))
    ups = [{"model": host_row(i)} for i in range(n_cpu)]
    cts = [int(c) for c in counts[:n_cpu]]
    state = {"cur": {"model": base0.clone()}, "m": {}, "v": {}}

    def one_round():
        agg, running = {"model": base0.clone()}, 0
        for w, c in zip(ups, cts):
            running += c
            torch_cpu.fedavg_round(agg, [w], [c], running)
            if fedopt:
                state["cur"] = torch_cpu.fedopt_adapt(sort, agg, state["cur"], state["m"], state["v"],
                                                      0.9, 0.99, 1e-2, 1e-3)
    try:
        one_round()
        ts = []
        for _ in range(rounds):
            t0 = time.perf_counter()
            one_round()
            ts.append(time.perf_counter() - t0)
    finally:
        torch.set_num_threads(prev)
    t = statistics.median(ts)
    ops = "FedAvg.do per arrival (fedavg.py:84-104)" + (
        f" + the {sort} step (fedopt.py:102-129)" if fedopt else "")
    return {
        "value": n_cpu * P / t, "unit": "client-params/s", "cores": cores, "kind": "port",
        "sample": f"reference eager round op sequence: {ops}, torch CPU (oracle/torch_cpu.py), the first "
                  f"{n_cpu} of the {n} arrivals x {P} {str(base0.dtype).replace('torch.', '')} params, median "
                  f"of {rounds} rounds ({t:.3f} s per {n_cpu} arrivals), {cores} threads on {_cpu_model()}; "
                  f"value = sampled arrival-params / time (the op sequence costs the same per arrival)",
        "host": env,
    }


def cpu_baseline_hier(rows, P, stale, rnd, rounds):
    """One middle aggregator of config 5 on host cores: FedBuff per arrival
    (fedbuff.py:94-96,136-157) + scale_add (:122-127) + the middle's delta
    (asyncfl/middle_aggregator.py:221-226, common/util.py:152-159)."""
    from oracle import torch_cpu
    C = len(rows)
    ts = []
    for _ in range(rounds):
        base = {"model": rows[0].clone()}
        t0 = time.perf_counter()
        agg = None
        for t in range(C):
            agg = torch_cpu.fedbuff_step(agg, {"model": rows[t]}, rnd, rnd - stale[t])
        prev = {"model": base["model"].clone()}
        torch_cpu.fedbuff_scale_add(base, agg, C)
        _ = {k: base[k] - prev[k] for k in base}
        ts.append(time.perf_counter() - t0)
    t = statistics.median(ts)
    return {
        "value": C * P / t, "unit": "client-params/s", "cores": torch.get_num_threads(), "kind": "port",
        "sample": f"one middle aggregator: reference FedBuff op sequence over {C} arrivals x {P} bf16 params "
                  f"+ scale_add + delta (torch CPU, oracle/torch_cpu.py), median of {rounds} ({t:.3f} s), "
                  f"{torch.get_num_threads()} threads on {_cpu_model()}",
    }


SETTLE = None   # what settle_hbm() saw before the timed region (every bench line reports it)


def settle_hbm(min_s: float = 7.0, window_s: float = 2.0, every_s: float = 0.25, tol: float = 0.015,
               max_s: float = 30.0, gb: float = 8.0):
    """Wait out another process's teardown before timing ("Cross-process spread"):
    after a process holding G GB exits, HBM reads run ~3.5 % slower for about G / 45 GB/s seconds
    (the driver wiping the freed memory: 1.4 s after 100 GB, 5.6 s after 250 GB,
    `profiles/r04tr_*.log`), and a bench's whole GPU phase fits inside that window.  Reads a
    ``gb`` scratch buffer with the 2-per-CU region probe every ``every_s`` for at least ``min_s``
    (a full 288 GB GPU's wipe) and until the readings of the last ``window_s`` agree within
    ``tol`` (at most ``max_s``).  None of the workload runs meanwhile, and nothing is freed to the
    driver (the block stays in torch's cache).  The readings go into the bench line."""
    global SETTLE
    buf = torch.empty(int(gb * 1e9) // 4, dtype=torch.float32, device="cuda")
    buf.fill_(1.0)
    t0 = time.perf_counter()
    need = max(2, int(round(window_s / every_s)) + 1)
    series = []
    while True:
        _, res = read_ceiling(buf, reps=3)
        r = res.get("region_1MiB_2perCU_6ld") if res else None
        if r is None:      # no probe library: nothing to settle on
            break
        t = time.perf_counter() - t0
        series.append((round(t, 2), round(r)))
        last = [v for _, v in series[-need:]]
        if t >= min_s and len(series) >= need and max(last) / min(last) - 1 < tol:
            break
        if t >= max_s:
            break
        time.sleep(every_s)
    del buf
    SETTLE = {"waited_s": round(time.perf_counter() - t0, 2), "probe_GBps": series,
              "rule": f"{gb:g} GB region-read probe every {every_s} s for >= {min_s} s, until {window_s} s of "
                      f"readings agree within {tol * 100:g} % (cap {max_s} s)"}
    return SETTLE


def timed(world, steps, warmup, step):
    from flame_amd import engine
    if SETTLE is None and torch.cuda.is_available() and os.environ.get("FLAME_BENCH_SETTLE", "1") != "0":
        settle_hbm()
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    engine.kernel_events = []
    from flame_amd import shard
    if shard.GATHER_TIMING is not None:      # the N>1 lines time the timed steps' gathers only
        shard.GATHER_TIMING.clear()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    global ISSUE_S
    ISSUE_S = time.perf_counter() - t0   # host time to issue the steps (GPU runs behind)
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    events = engine.kernel_events
    engine.kernel_events = None
    if world > 1:
        import torch.distributed as dist
        dev = "cpu" if dist.get_backend() == "gloo" else "cuda"
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, events


def kernel_stats(events, name):
    ks = [(e0.elapsed_time(e1) / 1e3, nb) for (nm, e0, e1, nb) in events if nm == name]
    if not ks:
        return None
    total_t = sum(t for t, _ in ks)
    total_b = sum(b for _, b in ks)
    return {"launches": len(ks), "avg_s": total_t / len(ks), "bytes_per_launch": total_b / len(ks),
            "achieved_GBps": total_b / total_t / 1e9}


def read_ceiling(buf: torch.Tensor, reps: int = 5, regions=()):
    """Same-device HBM streaming-read ceiling over an existing buffer (tools/hbm_probe.hip):
    the best of a grid-stride read (16,384 workgroups, 16 nt dwordx4 loads in flight per
    lane) and region-streaming reads (each workgroup one contiguous 1 MiB region -- the product
    kernel's access pattern with the fastest region size measured -- at full residency with 16
    loads per lane, and at 2 workgroups per CU with 6, the faster of the two since round 3).
    ``regions``: further region sizes (bytes) to probe the same way, e.g. a kernel's own
    per-workgroup region when it differs from 1 MiB.  Returns (best GB/s, {probe: GB/s})."""
    import ctypes
    import subprocess
    so = os.path.join(ROOT, "build", "hbm_probe.so")
    try:
        if not os.path.exists(so):
            os.makedirs(os.path.dirname(so), exist_ok=True)
            subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC",
                                   "-o", so, os.path.join(ROOT, "tools", "hbm_probe.hip")])
        L = ctypes.CDLL(so)
        L.probe_read_region.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
                                        ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]
    except Exception:  # noqa: BLE001
        return None, {}
    L.probe_read.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                             ctypes.c_void_p]
    nbytes = buf.numel() * buf.element_size() // (1 << 20) * (1 << 20)
    out = torch.zeros(4, dtype=torch.int32, device=buf.device)
    st = torch.cuda.current_stream(buf.device).cuda_stream
    probes = {
        "grid_stride_16384wg_16ld": lambda: L.probe_read(buf.data_ptr(), nbytes, out.data_ptr(), 16384, 2, st),
        "region_1MiB_16ld": lambda: L.probe_read_region(buf.data_ptr(), nbytes, out.data_ptr(), 1 << 20, 1 << 20,
                                                        16, st),
    }
    for r in regions:
        probes[f"region_{r >> 20}MiB_16ld"] = (lambda r=r: L.probe_read_region(buf.data_ptr(), nbytes, out.data_ptr(),
                                                                             r, r, 16, st))
    # the same region streams at 2 workgroups per CU (64 KiB of dynamic LDS each) with 6 loads in
    # flight per lane: the residency HBM reads fastest at (tools/occ_probe.py), the one the product
    # kernels now run at (flame_agg_reduce's FLAME_LO_CU path, FedOPT, the hierarchy kernel)
    if hasattr(L, "probe_read_region_persist"):
        L.probe_read_region_persist.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
                                                ctypes.c_int, ctypes.c_int64, ctypes.c_int,
                                                ctypes.POINTER(ctypes.c_int), ctypes.c_void_p]
        for r in (1 << 20, *regions):
            probes[f"region_{r >> 20}MiB_2perCU_6ld"] = (
                lambda r=r: L.probe_read_region_persist(buf.data_ptr(), nbytes // r * r, out.data_ptr(), r, 6, 0,
                                                        65536, None, st))
    res = {}
    for name, launch in probes.items():
        ts = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            if launch() != 0:
                return None, {}
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / 1e3)
        res[name] = nbytes / statistics.median(ts) / 1e9
    return max(res.values()), res


def make_clients(args, n, P, rank, dev, dtype=torch.float32):
    """n synthetic client updates of P params in HBM (tiled slab or one row each): the fp32
    synthetic values, rounded to ``dtype`` for a 16-bit model."""
    from flame_amd import engine
    tmp = torch.empty(P, dtype=torch.float32, device=dev)
    if args.layout == "slab":
        from flame_amd.slab import UpdateSlab
        store = UpdateSlab({"model": torch.empty(P, dtype=dtype)}, capacity=n, device=dev)
        client_w = []
        for i in range(n):
            engine.synth_fill_(tmp, args.seed, 1 + i + rank * 100_000, 0, 1e-2)
            client_w.append(store.put({"model": tmp.to(dtype)}))   # tiled slot views, held for the run
        del tmp
        return client_w, store.storage[dtype], (lambda i: store.read(i, "model").cpu())
    slab = torch.empty((n, P), dtype=dtype, device=dev)
    for i in range(n):
        engine.synth_fill_(tmp, args.seed, 1 + i + rank * 100_000, 0, 1e-2)
        slab[i].copy_(tmp)
    del tmp
    return [{"model": slab[i]} for i in range(n)], slab, (lambda i: slab[i].cpu())


def bench_feddyn_scaffold(args, world, rank, dev, n, P, client_w, base, counts):
    """FedDyn (feddyn.py:70-139) / SCAFFOLD (scaffold.py:92-150) server rounds through the
    drop-ins: every trainer active each round, updates (and SCAFFOLD control variates)
    resident in HBM.  Reports the round's kernels priced by their algorithmic bytes."""
    from flame_amd.optimizers import optimizer_provider
    keys = [f"{i:05d}" for i in range(n)]
    if args.workload == "feddyn":
        opt = optimizer_provider.get("feddyn", alpha=0.01, history=args.feddyn_history)
        # the role's active_ends are the channel's join order (feddyn/top_aggregator.py:137);
        # "shuffled" makes it differ from the cache's sorted order (two-phase program)
        ends = list(keys)
        if args.feddyn_order == "shuffled":
            ends = [keys[i] for i in np.random.default_rng(5).permutation(n)]
    else:
        opt = optimizer_provider.get("scaffold", k=3)
        opt.save_state("pre", dataset_sizes={k: int(c) for k, c in zip(keys, counts)},
                       glob_weights={"model": base})
    state = {"weights": {"model": base}}

    def step():
        cache = Cache()
        for i, k in enumerate(keys):
            cache[k] = TR(client_w[i], int(counts[i]))
        if args.workload == "feddyn":
            opt.save_state("pre", active_ends=ends)   # the role's per-round call (feddyn top_aggregator)
            state["weights"] = opt.do({"model": state["weights"]["model"].clone()}, cache, total=n)
        else:
            ctl = Cache()
            for i, k in enumerate(keys):    # control variates: the same synthetic tensors stand in
                ctl[k] = TR(client_w[n - 1 - i], 1)
            state["weights"] = opt.do({"model": state["weights"]["model"].clone()}, cache, total=n,
                                      control_cache=ctl)

    step()  # FedDyn: the first round copies every trainer's history (untimed, as FedOPT's round 1)
    elapsed, events = timed(world, args.steps, args.warmup, step)
    kname = "flame_feddyn_round" if args.workload == "feddyn" else "flame_agg_reduce"
    ks = kernel_stats(events, kname)
    if rank == 0:
        k_time = ks["avg_s"] * ks["launches"] / args.steps
        k_bytes = ks["bytes_per_launch"] * ks["launches"] / args.steps
        traffic, traffic_source = traffic_lookup(args.traffic, kernel=kname, clients=n, params=P,
                                                 workload=args.workload)
        print(json.dumps({
            "metric": f"aggregated params/sec (device-resident), {args.workload} server round",
            "value": n * P * world / (elapsed / args.steps), "unit": "client-params/s", "n_gpus": world,
            "steps": args.steps, "ms_per_step": elapsed / args.steps * 1e3, "dtype": "f32", "settle": SETTLE,
            "config": {"workload": f"{args.workload}: {n} clients x {P} fp32 params, {args.layout} layout"
                                   + (f", active_ends {args.feddyn_order}, {args.feddyn_history} histories"
                                      if args.workload == "feddyn" else "")},
            "roofline": {"bound": "hbm", "achieved": k_bytes / k_time / 1e9, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": k_bytes / k_time / 1e9 / PEAK_HBM_GBS, "kernel": kname,
                         "kernel_ms_per_step": k_time * 1e3, "launches_per_step": ks["launches"] / args.steps,
                         "algorithmic_bytes_per_step": k_bytes, "traffic_per_launch": traffic,
                         "traffic_source": traffic_source,
                         "bytes_per_client_param": k_bytes / (n * P * 4)},
        }), flush=True)


def traffic_lookup(path, **match):
    """HBM bytes per launch from the PMC-derived table (tools/pmc_traffic.py writes it from separate
    rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs): the LAST entry whose fields equal ``match``
    (``None`` in ``match`` = the field is absent or anything; a missing entry field counts as its
    given default), with where the bytes came from -- a lookup, not this run's counters."""
    try:
        entries = json.load(open(path))
        entries = entries["entries"] if "entries" in entries else [entries]
    except Exception:  # noqa: BLE001
        return None, None
    hit = None
    for tr in entries:
        if all(v is None or tr.get(k, _TRAFFIC_DEFAULTS.get(k)) == v for k, v in match.items()):
            hit = tr
    if hit is None:
        return None, None
    return hit["hbm_bytes_per_launch"], {
        "kind": "lookup", "file": os.path.relpath(path, ROOT),
        "entry": {k: hit.get(k) for k in ("kernel", "clients", "params", "layout", "workload")},
        "counters": hit.get("source", "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (source not recorded in "
                                      "this entry)"),
        "traffic_over_algorithmic": hit.get("traffic_over_algorithmic")}


_TRAFFIC_DEFAULTS = {"layout": "row"}
DTYPES = {"f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16}


def bench_eager(args, world, rank, dev, n, P, client_w, base, counts, host_row=None):
    """The eager top aggregator's round (eager_syncfl/top_aggregator.py:36-90) on
    device-resident updates: base = deepcopy(weights), then one do() per arrival with the
    running total; the role keeps the returned object (read once, at the round's end).
    fedavg_eager: --eager-defer on: FedAvg(defer=True), one launch per round; off: one per
    arrival.  fed{adam,yogi,adagrad}_eager: FedOPT.do per arrival (FedAvg of the arrival + the
    adaptive step); --eager-defer on: FedOPT(defer=True) queues the calls and runs the round as
    ONE flame_fedopt_chain launch when the role reads the result; off: one fused
    flame_fedopt_reduce_adapt launch per arrival.  The first round -- untimed, reported apart --
    holds the round-1 passthrough and the aliased step (current_weights IS base:
    FLAME_SEG_CUR_IS_AVG)."""
    from flame_amd import engine
    from flame_amd.optimizers import optimizer_provider
    if world > 1:
        raise SystemExit(f"--workload {args.workload} is a one-GPU bench")
    defer = args.eager_defer == "on"
    sort = args.workload[:-len("_eager")]
    fedopt = sort != "fedavg"
    opt = optimizer_provider.get(sort, defer=defer)
    kname = ("flame_fedopt_chain" if defer else "flame_fedopt_reduce_adapt") if fedopt else "flame_agg_reduce"
    keys = [f"{i:05d}" for i in range(n)]
    state = {"weights": {"model": base}}
    base0 = base.cpu() if (rank == 0 and args.cpu_clients > 0 and host_row is not None) else None
    dt = args.dtype
    isz = base.element_size()

    def step():
        bw = {"model": state["weights"]["model"].clone()}      # deepcopy(self.weights)
        running, out = 0, None
        for i, k in enumerate(keys):
            running += int(counts[i])
            cache = Cache()
            cache[k] = TR(client_w[i], int(counts[i]))
            out = opt.do(bw, cache, total=running, num_trainers=n)
        state["weights"] = {"model": out["model"]}              # self.weights = global_weights; read

    first = None
    if fedopt:
        engine.kernel_events = []
        step()                  # round 1: passthrough, then the aliased step, then the rest
        torch.cuda.synchronize()
        ev = [e for e in engine.kernel_events if e[0] == kname]
        engine.kernel_events = None
        first = {"launches": len(ev), "first_launch_kernel_ms": ev[0][1].elapsed_time(ev[0][2]) if ev else None,
                 "note": "arrival 1: FedAvg passthrough (flame_agg_reduce); arrival 2: current IS base, the "
                         "step with FLAME_SEG_CUR_IS_AVG; " + ("arrivals 2..n: one flame_fedopt_chain launch"
                                                               if defer else "arrivals 3..n: fused, one launch each")}
    elapsed, events = timed(world, args.steps, args.warmup, step)
    ks = kernel_stats(events, kname)
    if rank == 0:
        k_time = ks["avg_s"] * ks["launches"] / args.steps
        k_bytes = ks["bytes_per_launch"] * ks["launches"] / args.steps
        # that variant's (and dtype's) entry or None
        traffic, traffic_source = traffic_lookup(args.traffic, kernel=kname, clients=n, params=P,
                                                 workload=args.workload + ("" if dt == "f32" else f"_{dt}"))
        cpu = (cpu_baseline_eager(sort, host_row, n, P, base0, counts, min(args.cpu_clients, 8), args.cpu_rounds)
               if base0 is not None else None)
        print(json.dumps({
            "metric": f"aggregated params/sec (device-resident), eager {sort} round",
            "value": n * P / (elapsed / args.steps), "unit": "client-params/s", "n_gpus": world,
            "steps": args.steps, "ms_per_step": elapsed / args.steps * 1e3, "dtype": dt, "settle": SETTLE,
            "config": {"workload": f"{args.workload}: {n} arrivals (one do() each, running total) x {P} {dt} "
                                   f"params, {args.layout} layout, defer {args.eager_defer}"},
            "first_round": first,
            "roofline": {"bound": "hbm", "achieved": k_bytes / k_time / 1e9, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": k_bytes / k_time / 1e9 / PEAK_HBM_GBS, "kernel": kname,
                         "kernel_ms_per_step": k_time * 1e3, "launches_per_step": ks["launches"] / args.steps,
                         "algorithmic_bytes_per_step": k_bytes, "traffic_per_launch": traffic,
                         "traffic_source": traffic_source,
                         "bytes_per_client_param": k_bytes / (n * P * isz),
                         **({"note": "flame_fedopt_chain runs every arrival's adaptive step in sequence per "
                                     "element (~18 VALU instructions each with the fast correctly rounded "
                                     "sqrt and divide, 2 of them quarter-rate transcendentals): VALU and "
                                     "HBM both ~70-75 % busy (DESIGN.md §4)"}
                            if fedopt and defer and dt == "f32" else
                            {"note": f"flame_fedopt_chain, {dt}: every op rounded to {dt} as torch-CPU does, on "
                                     f"packed fp32 with one-instruction roundings (DESIGN.md §4): VALU-bound at "
                                     f"2 bytes per element"}
                            if fedopt and defer else {})},
            "cpu_baseline": cpu,
        }), flush=True)


def launch_plan(gpus, env):
    """What ``bench.py --gpus N`` does in this process, decided before anything touches the GPU.

    ("run", None)    this process is one rank: torchrun's env names the world (and it equals
                     --gpus), or N == 1 with no launcher;
    ("spawn", N)     N > 1 and no launcher env: start N ranks under torch.distributed.run;
    ("error", msg)   the launcher's world and --gpus disagree, or N < 1.
    Every rank returns the full model (syncfl/top_aggregator.py:161-173), so N is the number of
    GPUs the line is measured on -- never silently fewer."""
    if gpus < 1:
        return "error", f"bench.py: --gpus {gpus}: need at least one GPU"
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != gpus:
            return "error", (f"bench.py: --gpus {gpus} but the launcher's WORLD_SIZE is {ws}: "
                             f"run with --gpus {ws} or launch {gpus} ranks")
        return "run", None
    if "RANK" in env or gpus == 1:
        return "run", None
    return "spawn", gpus


def spawn_ranks(gpus, argv):
    """Start ``gpus`` ranks of this script under torch.distributed.run (fresh child processes:
    this parent has not initialised the GPU and never execs), relay their stdout line by line
    (rank 0's JSON line included) and return the launcher's exit code (non-zero when any rank
    failed)."""
    import socket
    import subprocess
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ, FLAME_BENCH_LAUNCHER=f"bench.py --gpus {gpus} -> torch.distributed.run")
    print(f"bench.py: --gpus {gpus} without a launcher: starting {gpus} ranks: {' '.join(cmd)}",
          file=sys.stderr, flush=True)
    proc = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True, bufsize=1)
    for line in proc.stdout:
        sys.stdout.write(line)
        sys.stdout.flush()
    return proc.wait()


def launcher(world):
    """How this line's ranks were started (the driver's own torchrun, bench.py --gpus N, or none)."""
    return os.environ.get("FLAME_BENCH_LAUNCHER",
                          "torch.distributed.run" if "WORLD_SIZE" in os.environ else "single process")


def main():
    args = parse()
    what, arg = launch_plan(args.gpus, os.environ)
    if what == "error":
        raise SystemExit(arg)
    if what == "spawn":
        raise SystemExit(spawn_ranks(arg, sys.argv[1:]))
    if args.dtype != "f32" and (args.e2e or not args.workload.endswith("_eager")):
        raise SystemExit(f"--dtype {args.dtype}: the fed*_eager workloads only (--workload {args.workload} runs its "
                         f"BASELINE config's dtype)")
    world, rank, local = setup_dist(args.force_shard)
    dev = torch.device("cuda", local)
    from flame_amd import _native, engine, synth
    from flame_amd.optimizers import optimizer_provider
    _native.lib()  # the HIP library is required; no fallback

    if args.workload == "hier_fedbuff":
        return bench_hier(args, world, rank, dev)
    if args.workload == "fedbuff":
        return bench_fedbuff(args, world, rank, dev)

    n = args.clients or {"feddyn": 512, "scaffold": 512}.get(args.workload,
                                                          64 if args.workload.endswith("_eager") else 1024)
    P = args.params or 25_000_000
    # ---- synthetic inputs (counter generator; rank-specific streams)
    if args.e2e:
        if args.e2e_mode == "shm_shard" or (world > 1 and args.e2e_mode == "shm"):
            return bench_e2e_shm_sharded(args, world, rank, dev, n, P)
        if world > 1:
            raise SystemExit(f"--e2e at {world} GPUs: --e2e-mode shm (the sharded shm ingest); "
                             f"{args.e2e_mode} is a one-GPU mode")
        return bench_e2e(args, n, P, dev)
    if (world > 1 or args.force_shard) and args.workload in ("fedavg", "fedadam", "fedyogi", "fedadagrad"):
        return bench_sharded(args, world, rank, dev, n, P)
    dtype = DTYPES[args.dtype]
    client_w, slab_buf, host_row = make_clients(args, n, P, rank, dev, dtype)
    base = torch.empty(P, dtype=torch.float32, device=dev)
    engine.synth_fill_(base, args.seed, rank * 100_000, 0, 1.0)
    base = base.to(dtype)
    counts = synth.counts(args.seed, n)
    if args.workload in ("feddyn", "scaffold"):
        return bench_feddyn_scaffold(args, world, rank, dev, n, P, client_w, base, counts)
    if args.workload.endswith("_eager"):
        return bench_eager(args, world, rank, dev, n, P, client_w, base, counts,
                           host_row if world == 1 else None)
    base0 = base.clone() if (rank == 0 and world == 1 and args.cpu_clients > 0) else None
    total = int(counts.sum())
    keys = [f"{i:05d}" for i in range(n)]
    torch.cuda.synchronize()

    if world > 1:
        raise SystemExit(f"--workload {args.workload} has no multi-GPU bench (its drop-in shards via "
                         f"flame_amd.shard.ShardedOptimizer; see tests/test_shard_gloo.py)")
    opt = optimizer_provider.get(args.workload)
    state = {"weights": {"model": base}}

    def received():
        # the role's cache of received TrainResults (syncfl/top_aggregator.py:136-157): built as
        # the updates arrive, before the aggregation starts -- like the CPU baseline, which
        # times the reference's op sequence over already-received updates
        cache = Cache()
        for i, k in enumerate(keys):
            cache[k] = TR(client_w[i], int(counts[i]))
        return cache
    arrived = [received() for _ in range(args.warmup + args.steps + (1 if args.workload != "fedavg" else 0))]

    def step():
        cache = arrived.pop()
        if args.workload == "fedavg":
            opt.do(state["weights"], cache, total=total, num_trainers=n)
        else:  # FedOPT caller convention: weights = do(deepcopy(weights), ...)
            state["weights"] = opt.do({"model": state["weights"]["model"].clone()}, cache, total=total,
                                      num_trainers=n)

    if args.workload != "fedavg":
        step()  # FedOPT round 1 is a passthrough (fedopt.py:87-88); time adaptive rounds only
    elapsed, events = timed(world, args.steps, args.warmup, step)
    name = "flame_agg_reduce" if args.workload == "fedavg" else "flame_fedopt_reduce_adapt"
    ks = kernel_stats(events, name)

    if rank == 0:
        traffic, traffic_source = traffic_lookup(args.traffic, kernel=name, clients=n, params=P, layout=args.layout,
                                                 workload=args.workload)
        cpu = None
        if world == 1 and args.cpu_clients > 0 and args.workload == "fedavg":
            cpu = cpu_baseline(host_row, n, P, base0, counts, args.cpu_clients, args.cpu_rounds)
        elif world == 1 and args.cpu_clients > 0:
            cpu = cpu_baseline_fedopt(args.workload, host_row, n, P, base0, counts, args.cpu_clients,
                                      args.cpu_rounds)
        # (the kernel's own per-workgroup region too: n x 4 KiB of the tiled slab)
        ceiling, probes = (read_ceiling(slab_buf, regions=(n * 4096,) if args.layout == "slab" and n * 4096 != 1 << 20
                                        else ()) if world == 1 else (None, {}))
        # a piece-pipelined step has several launches: price the step's kernels as one
        launches_per_step = ks["launches"] / args.steps
        k_time = ks["avg_s"] * launches_per_step
        k_bytes = ks["bytes_per_launch"] * launches_per_step
        achieved = k_bytes / k_time / 1e9
        line = {
            # BASELINE.json's metric for the headline FedAvg; the FedOPT workloads (config 4) name theirs
            "metric": METRIC if args.workload == "fedavg" else
            f"aggregated params/sec (device-resident), {n}-client "
            f"{ {'fedadam': 'FedAdam', 'fedyogi': 'FedYogi', 'fedadagrad': 'FedAdaGrad'}.get(args.workload, args.workload)}"
            f" (adaptive round)",
            "value": n * P * world / (elapsed / args.steps),
            "unit": "client-params/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "host_issue_ms_per_step": ISSUE_S / args.steps * 1e3, "settle": SETTLE,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (counter-based generator, flame_amd/synth.py), resident in HBM",
            "config": {
                "workload": f"{args.workload}: {n} clients x {P} fp32 params per GPU, {args.layout} layout"
                            + (f" (model {P * world} params, parameter-sharded, RCCL all-gather"
                               f"{' pipelined' if (args.workload == 'fedavg' and not args.no_overlap) else ''})"
                               if world > 1 else ""),
                "clients": n, "params_per_gpu": P, "global_params": P * world,
                "parallelism": f"param-shard{world}" if world > 1 else "single",
            },
            "roofline": {
                "bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": achieved / PEAK_HBM_GBS, "traffic": traffic, "traffic_source": traffic_source,
                "kernel": name, "kernel_ms": k_time * 1e3, "algorithmic_bytes": k_bytes,
                "launches_per_step": launches_per_step,
                # same device, same buffer: plain streaming-read probe (tools/hbm_probe.hip)
                "measured_read_ceiling_GBps": ceiling, "read_probes_GBps": probes,
                "frac_of_measured_ceiling": (achieved / ceiling) if ceiling else None,
            },
            "cpu_baseline": cpu,
            "launcher": launcher(world),
        }
        print(json.dumps(line), flush=True)
    import torch.distributed as dist
    if dist.is_initialized():
        dist.destroy_process_group()


def _local_slab(plan, n, dev, seed, sigma):
    """n synthetic client updates holding only this rank's slices of the (global) model: a
    tiled slab over the plan's local names, as DeviceUpdateCache(shard=plan) writes it.  The
    counter generator is indexed by GLOBAL element, so every rank holds slices of one model."""
    from flame_amd import engine
    from flame_amd.slab import UpdateSlab
    store = UpdateSlab(plan.local_template(), capacity=n, device=dev)
    tmp = {nm: torch.empty(plan.local_numel[nm], dtype=plan.dtypes[plan.by_name[nm].key], device=dev)
           for nm in plan.names}
    ws = []
    for i in range(n):
        for sub in plan.subs:
            engine.synth_fill_(tmp[sub.name], seed, 1 + i, sub.lo, sigma)
        ws.append(store.put(tmp))
    return store, ws


def _fracs(args, shard, default=None):
    if args.no_overlap:
        return (1.0,)
    if args.shard_fracs:
        return tuple(float(x) for x in args.shard_fracs.split(","))
    return default or shard.DEFAULT_FRACS


def _collective_note(plan, world, itemsize):
    from flame_amd import shard
    recv = sum((s.g1 - s.g0) - (s.hi - s.lo) for s in plan.subs if not s.tail) * itemsize
    return {"kind": "in-place all_gather_into_tensor per wave (RCCL over xGMI)" if world > 1 else "none (world 1)",
            "waves": plan.n_waves, "bytes_received_per_rank": recv,
            # which torch.distributed calls the gathers took (flame_amd.shard.GATHER_STATS): "async" =
            # the public all_gather_into_tensor per piece, "coalesced" = torch's _coalescing_manager group
            # (a wave of several same-dtype pieces), "host_staged" = gloo with CUDA tensors
            "gather_calls": dict(shard.GATHER_STATS),
            "wave_elements_per_rank": [sum(s.hi - s.lo for s in plan.subs if s.wave == w and not s.tail)
                                       for w in range(plan.n_waves)],
            "replicated_tail_elements": sum(s.hi - s.lo for s in plan.subs if s.tail)}


# ------------------------------------------------------------------ N>1 self-check (untimed)
# Run after the timed steps of every parameter-sharded line: each rank digests the full model
# it holds (every rank must end with the whole model, syncfl/top_aggregator.py:161-173), the
# digests are all-gathered and compared, and sampled global elements of every wave (plus
# every rank boundary and the replicated tails) are recomputed on the host from the counter
# generator with the reference's per-op roundings (numpy fp32 ops round once each, no FMA;
# bf16 through flame_amd.synth's RNE) and compared bitwise on every rank.
def _bf16(x):
    from flame_amd import synth
    return synth.bf16_bits_to_f32(synth.f32_to_bf16_bits(np.asarray(x, dtype=np.float32)))


def _rate32(r):
    return np.float32(r)


def sample_indices(plan, key, per_wave=64, seed=0):
    """~per_wave global element indices of ``key`` per wave, every rank boundary of every
    piece, and the key's tail (replicated on every rank)."""
    rng = np.random.default_rng(seed)
    world = plan.world
    picks = []
    for w in range(plan.n_waves):
        pieces = [(s.g0, s.g1) for s in plan.subs if s.key == key and s.wave == w and not s.tail]
        if not pieces:
            continue
        sizes = np.array([b - a for a, b in pieces], dtype=np.int64)
        pos = rng.integers(0, int(sizes.sum()), size=per_wave)
        ends = np.cumsum(sizes)
        for p in pos:
            j = int(np.searchsorted(ends, p, side="right"))
            picks.append(pieces[j][0] + int(p - (ends[j] - sizes[j])))
        for a, b in pieces:
            per = (b - a) // world
            for r in range(world):
                picks += [a + r * per, a + (r + 1) * per - 1]
    for s in plan.subs:
        if s.key == key and s.tail and s.g1 > s.g0:
            picks += list(range(s.g0, min(s.g1, s.g0 + per_wave)))
    return np.unique(np.asarray(picks, dtype=np.int64))


def host_fedavg_rounds(seed, counts, idx, rounds, base=None):
    """FedAvg.do (fedavg.py:79-104) ``rounds`` times in place over the n synthetic clients."""
    from flame_amd import synth
    total = int(np.asarray(counts).sum())
    r32 = [_rate32(int(c) / total) for c in counts]
    acc = synth.synth_f32(seed, 0, idx, 1.0) if base is None else base
    cl = [synth.synth_f32(seed, 1 + i, idx, 1e-2) for i in range(len(counts))]
    for _ in range(rounds):
        for v, r in zip(cl, r32):
            acc = acc + v * r
    return acc


def host_fedopt_rounds(sort, hyper, seed, counts, idx, rounds):
    """FedOPT.do (fedopt.py:58-129) from the synthetic base: round 1 the FedAvg passthrough,
    then FedAvg of (a copy of) current + the adaptive step, every op rounded in fp32."""
    from flame_amd import synth
    b1, omb1, b2, omb2, eta, tau = [np.float32(x) for x in hyper]
    cur = synth.synth_f32(seed, 0, idx, 1.0)
    m = v = None
    for r in range(rounds):
        avg = host_fedavg_rounds(seed, counts, idx, 1, base=cur.copy())
        if r == 0:
            cur = avg
            continue
        if m is None:
            m, v = np.zeros_like(avg), np.zeros_like(avg)
        d = avg - cur
        m = b1 * m + omb1 * d
        d2 = d * d
        if sort == "fedadam":
            v = b2 * v + omb2 * d2
        elif sort == "fedyogi":
            v = v - (omb2 * d2) * np.sign(v - d2).astype(np.float32)
        else:
            v = v + d2
        cur = cur + (eta * m) / (np.sqrt(v) + tau)
    return cur


def host_hier_rounds(seed, M, C, idx, rounds, rnd, fetched, sync):
    """Config 5's round ``rounds`` times in bf16: every middle's FedBuff over its C arrivals
    (fedbuff.py:94-96,136-157) + scale_add + delta (asyncfl/middle_aggregator.py:221-226,246),
    the top's FedBuff over the deltas (rate 1/sqrt(1 + m % 2)) + scale_add (top_goal M); sync:
    every middle's FedAvg from its weights, delta, the top's FedAvg of the deltas
    (syncfl/middle_aggregator.py:163-229, syncfl/top_aggregator.py:122-176)."""
    import math
    from flame_amd import synth
    cnt = synth.counts(seed, M * C)
    stale = [int(x) % 4 for x in cnt]
    gw = _bf16(synth.synth_f32(seed, 0, idx, 1.0))
    mids = [gw.copy() for _ in range(M)]
    shared = gw.copy()
    arr = [_bf16(synth.synth_f32(seed, 1 + i, idx, 1e-2)) for i in range(M * C)]
    for _ in range(rounds):
        if sync:
            totals = [int(cnt[m * C:(m + 1) * C].sum()) for m in range(M)]
            top_total = sum(totals)
            for m in range(M):
                w = shared if fetched else mids[m]
                a = w
                for t in range(C):
                    i = m * C + t
                    a = _bf16(a + _bf16(arr[i] * _rate32(int(cnt[i]) / totals[m])))
                d = _bf16(a - w)
                if not fetched:
                    mids[m] = a
                gw = _bf16(gw + _bf16(d * _rate32(totals[m] / top_total)))
            continue
        top = None
        for m in range(M):
            w = shared if fetched else mids[m]
            a = None
            for t in range(C):
                i = m * C + t
                tmp = _bf16(arr[i] * _rate32(1 / math.sqrt(1 + stale[i])))
                a = tmp if a is None else _bf16(a + tmp)
            nw = _bf16(w + _bf16(a / np.float32(C)))
            d = _bf16(nw - w)
            if not fetched:
                mids[m] = nw
            tmp = _bf16(d * _rate32(1 / math.sqrt(1 + rnd - (rnd - m % 2))))
            top = tmp if top is None else _bf16(top + tmp)
        gw = _bf16(gw + _bf16(top / np.float32(M)))
    return gw


def verify_sharded(model: torch.Tensor, idx, expected) -> dict:
    """Digest of this rank's full model, all-gathered; the sampled elements vs the host
    restatement on every rank.  Returns the line's ``gather_check`` object."""
    import hashlib
    import torch.distributed as dist
    t = model.detach().contiguous().view(-1)
    h = hashlib.blake2b(t.view(torch.uint8).cpu().numpy(), digest_size=16).hexdigest()   # (no bytes copy)
    got = t[torch.as_tensor(idx, device=t.device)].cpu()
    if got.dtype == torch.bfloat16:
        gb = got.view(torch.int16).numpy().view(np.uint16)
        eb = np.asarray(__import__("flame_amd.synth", fromlist=["x"]).f32_to_bf16_bits(expected))
    else:
        gb = got.numpy().view(np.uint32)
        eb = np.asarray(expected, dtype=np.float32).view(np.uint32)
    bad = int(np.count_nonzero(gb != eb))
    digests, bads = [h], [bad]
    if dist.is_available() and dist.is_initialized():
        digests = [None] * dist.get_world_size()
        bads = [None] * dist.get_world_size()
        dist.all_gather_object(digests, h)
        dist.all_gather_object(bads, bad)
    return {"ranks_agree": len(set(digests)) == 1, "digest": digests[0], "rank_digests": digests,
            "sampled_elements": int(len(idx)), "sample_mismatches_per_rank": bads,
            "sample_parity": "bitwise" if not any(bads) else f"MISMATCH ({sum(bads)} sampled elements)"}


def _checked(gc) -> None:
    """A failed self-check fails the run (after the line is printed)."""
    if not gc["ranks_agree"] or any(gc["sample_mismatches_per_rank"]):
        raise SystemExit(f"bench.py: N>1 self-check failed: ranks_agree={gc['ranks_agree']}, "
                         f"sample mismatches per rank {gc['sample_mismatches_per_rank']}")


def bench_sharded(args, world, rank, dev, n, P):
    """Configs 3/4 at N GPUs through the product's ShardedOptimizer: weak scaling -- the
    model has P x world params; each rank owns P of them (plus the replicated key tails)
    and holds only its slices of the n client updates; every step = one FedAvg.do (or
    FedOPT adaptive round) on the full model dict, three waves of reductions with their
    in-place RCCL all-gathers overlapped behind the next wave."""
    from flame_amd import engine, shard, synth
    from flame_amd.optimizers import optimizer_provider
    G = P * world
    inner = optimizer_provider.get(args.workload)
    opt = shard.ShardedOptimizer(inner, device=dev, fracs=_fracs(args, shard))
    opt.set_layout({"model": torch.empty(G, dtype=torch.float32, device="meta")})
    plan = opt.plan
    store, client_w = _local_slab(plan, n, dev, args.seed, 1e-2)
    base = torch.empty(G, dtype=torch.float32, device=dev)
    engine.synth_fill_(base, args.seed, 0, 0, 1.0)
    counts = synth.counts(args.seed, n)
    total = int(counts.sum())
    keys = [f"{i:05d}" for i in range(n)]
    fedavg = args.workload == "fedavg"
    torch.cuda.synchronize()
    state = {"weights": {"model": base}}

    def received():
        cache = Cache()
        for i, k in enumerate(keys):
            cache[k] = TR(client_w[i], int(counts[i]))
        return cache
    arrived = [received() for _ in range(args.warmup + args.steps + (0 if fedavg else 1))]

    rounds = [0]

    def step():
        cache = arrived.pop()
        rounds[0] += 1
        if fedavg:        # syncfl top: FedAvg mutates the base in place (fedavg.py:74,87)
            opt.do(state["weights"], cache, total=total, num_trainers=n)
        else:             # FedOPT caller convention: weights = do(deepcopy(weights), ...)
            state["weights"] = opt.do({"model": state["weights"]["model"].clone()}, cache, total=total,
                                      num_trainers=n)

    if not fedavg:
        step()            # FedOPT round 1 is a passthrough (fedopt.py:87-88); time adaptive rounds only
    shard.GATHER_TIMING = []
    elapsed, events = timed(world, args.steps, args.warmup, step)
    gt, shard.GATHER_TIMING = shard.GATHER_TIMING, None
    name = "flame_agg_reduce" if fedavg else "flame_fedopt_reduce_adapt"
    ks = kernel_stats(events, name)
    attrib = time_attribution(world, ks["avg_s"] * ks["launches"] / args.steps * 1e3 if ks else None,
                              elapsed / args.steps * 1e3, gt)
    # untimed self-check: every rank holds the same full model, sampled elements == the host
    idx = sample_indices(plan, "model", seed=args.seed)
    if fedavg:
        expected = host_fedavg_rounds(args.seed, counts, idx, rounds[0])
    else:
        expected = host_fedopt_rounds(args.workload, engine.fedopt_scalars(inner.beta_1, inner.beta_2, inner.eta,
                                                                           inner.tau),
                                      args.seed, counts, idx, rounds[0])
    gc = verify_sharded(state["weights"]["model"], idx, expected)
    gc["rounds_checked"] = rounds[0]
    if rank == 0:
        lps = ks["launches"] / args.steps
        k_time, k_bytes = ks["avg_s"] * lps, ks["bytes_per_launch"] * lps
        achieved = k_bytes / k_time / 1e9
        # the per-rank shape's PMC bytes (n clients x P params, one launch): a lookup, labelled
        traffic, traffic_source = traffic_lookup(args.traffic, kernel=name, clients=n, params=P, layout="slab",
                                                 workload=args.workload)
        if traffic_source is not None:
            traffic_source["note"] = (f"measured on the unsharded per-rank shape (one launch); this line runs "
                                      f"{lps:g} launches per step over {plan.owned_elements()} owned params")
        print(json.dumps({
            "metric": METRIC if fedavg else f"aggregated params/sec (device-resident), {n}-client {args.workload} "
                                            f"(adaptive round)",
            "value": n * P * world / (elapsed / args.steps), "unit": "client-params/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
            "host_issue_ms_per_step": ISSUE_S / args.steps * 1e3, "settle": SETTLE, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (counter-based generator, flame_amd/synth.py), rank-local slices resident in HBM",
            "config": {"workload": f"{args.workload}: {n} clients x {G} fp32 params, parameter-sharded over "
                                   f"{world} rank(s) (flame_amd.shard.ShardedOptimizer, {plan.owned_elements()} "
                                   f"params per rank, tiled rank-local slab)",
                       "clients": n, "params_per_gpu": P, "global_params": G,
                       "parallelism": f"param-shard{world}"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": achieved / PEAK_HBM_GBS, "traffic": traffic, "traffic_source": traffic_source,
                         "kernel": name, "kernel_ms": k_time * 1e3, "algorithmic_bytes": k_bytes,
                         "launches_per_step": lps},
            "time_attribution": attrib,
            "collective": _collective_note(plan, world, 4),
            "process_group": process_group_info(),
            "launcher": launcher(world),
            "gather_check": gc,
            "cpu_baseline": None,
        }), flush=True)
    import torch.distributed as dist
    if dist.is_initialized():
        dist.destroy_process_group()
    _checked(gc)


def _middle_arrivals(args, M, C, client_w, stale, rnd):
    """The middles' arrivals of one round (asyncfl/middle_aggregator.py:164-203): each arrival
    is a TrainResult (count 1, version rnd - staleness) the middle role builds from its
    message; ``--hier-arrivals batched`` hands a middle's round to ONE
    ``FedBuff.do_arrivals`` call, ``per-do`` calls ``do()`` per arrival with a one-entry
    cache as the role does.  Returns the middles' aggregates."""
    def batched(mid_opts):
        return [mid_opts[m].do_arrivals(None, [TR(client_w[i], 1, rnd - stale[i]) for i in range(m * C, (m + 1) * C)],
                                        version=rnd) for m in range(M)]

    def per_do(mid_opts):
        aggs = [None] * M
        for m in range(M):
            opt = mid_opts[m]
            for t in range(C):
                i = m * C + t
                cache = Cache()
                cache[f"{i:05d}"] = TR(client_w[i], 1, rnd - stale[i])
                aggs[m] = opt.do(aggs[m], cache, total=1, version=rnd)
        return aggs
    return batched if args.hier_arrivals == "batched" else per_do


def bench_hier_sharded(args, world, rank, dev, M, C, P):
    """Config 5 as named (hierarchical FedBuff parameter-sharded over the node's GPUs with an
    RCCL all-gather) through the product's ShardedHierarchy: the model has P x world bf16
    params; each rank holds its slices of the M x C arrivals, of the 64 middles' weights and
    FedBuff aggregates and of the top aggregate; per step the middles' do() per arrival,
    then ShardedHierarchy.round (one flame_hier_fedbuff launch per wave) with the top model
    all-gathered in place wave by wave (sync mode: ShardedHierarchy.sync_round)."""
    from flame_amd import engine, shard, synth
    G, dt = P * world, torch.bfloat16
    if args.hier_mode not in ("fused", "sync"):
        raise SystemExit("multi-GPU hier bench: --hier-mode fused or sync (the product's ShardedHierarchy)")
    hier = shard.ShardedHierarchy({"model": torch.empty(G, dtype=dt, device="meta")}, device=dev,
                                  fracs=_fracs(args, shard, shard.HIER_FRACS),
                                  middles=M if args.hier_wave_quantum == "on" else None,
                                  sync=args.hier_mode == "sync")
    plan = hier.plan
    store, client_w = _local_slab(plan, M * C, dev, args.seed + 4, 1e-2)
    gw = torch.empty(G, dtype=dt, device=dev)
    engine.synth_fill_(gw, args.seed + 4, 0, 0, 1.0)
    fetched = args.hier_middles == "fetched"
    if fetched:   # every middle holds the model it fetched from the top (read-only)
        shared = {"model": gw.clone()}
        mids = [shared] * M
    else:         # each middle's own weights: sharded state, this rank's slices only
        own = collections.OrderedDict((nm, torch.empty(plan.local_numel[nm], dtype=dt, device=dev)) for nm in plan.names)
        for sub in plan.subs:
            engine.synth_fill_(own[sub.name], args.seed + 4, 0, sub.lo, 1.0)
        if args.hier_mid_layout == "tiled":     # the middles' weights as the slots of one tiled store
            from flame_amd.slab import UpdateSlab
            mid_store = UpdateSlab(plan.local_template(), capacity=M, device=dev)
            mids = [mid_store.put(own) for _ in range(M)]
        else:
            mids = [collections.OrderedDict((k, v.clone()) for k, v in own.items()) for _ in range(M)]
    stale = [int(x) % 4 for x in synth.counts(args.seed + 4, M * C)]
    counts = [int(c) for c in synth.counts(args.seed + 4, M * C)]
    rnd = 10
    mid_opts = [hier.middle_optimizer() for _ in range(M)]
    torch.cuda.synchronize()

    middle_arrivals = _middle_arrivals(args, M, C, client_w, stale, rnd)

    def step_fused():
        aggs = middle_arrivals(mid_opts)
        hier.round([(mids[m], aggs[m], C, rnd - (m % 2)) for m in range(M)], None, version=rnd,
                   top_weights={"model": gw}, top_goal=M, update_middle_weights=not fetched)

    def sync_specs():
        # every middle's cache of received updates (syncfl/middle_aggregator.py:136-160), filled
        # as the updates arrive -- before the aggregation starts, as in the FedAvg bench
        specs = []
        for m in range(M):
            cache = Cache()
            for t in range(C):
                i = m * C + t
                cache[f"{i:05d}"] = TR(client_w[i], counts[i])
            specs.append((mids[m], cache, sum(counts[m * C:(m + 1) * C])))
        return specs
    arrived = [sync_specs() for _ in range(args.warmup + args.steps)] if args.hier_mode == "sync" else []

    def step_sync():
        hier.sync_round(arrived.pop(), {"model": gw}, update_middle_weights=not fetched)

    rounds = [0]
    body = step_sync if args.hier_mode == "sync" else step_fused

    def step():
        rounds[0] += 1
        body()

    shard.GATHER_TIMING = []
    elapsed, events = timed(world, args.steps, args.warmup, step)
    gt, shard.GATHER_TIMING = shard.GATHER_TIMING, None
    ks = kernel_stats(events, "flame_hier_fedbuff")
    attrib = time_attribution(world, ks["avg_s"] * ks["launches"] / args.steps * 1e3 if ks else None,
                              elapsed / args.steps * 1e3, gt)
    idx = sample_indices(plan, "model", seed=args.seed)
    gc = verify_sharded(gw, idx, host_hier_rounds(args.seed + 4, M, C, idx, rounds[0], rnd, fetched,
                                                  args.hier_mode == "sync"))
    gc["rounds_checked"] = rounds[0]
    if rank == 0:
        lps = ks["launches"] / args.steps
        k_time, k_bytes = ks["avg_s"] * lps, ks["bytes_per_launch"] * lps
        sync = args.hier_mode == "sync"
        traffic, traffic_source = (traffic_lookup(args.traffic, kernel="flame_hier_fedbuff", clients=M * C, params=P,
                                                  layout="slab", workload="hier_fedbuff" if not fetched
                                                  else "hier_fedbuff_fetched") if not sync else (None, None))
        if traffic_source is not None:
            traffic_source["note"] = (f"measured on the unsharded per-rank shape (one launch); this line runs "
                                      f"{lps:g} launches per step over {plan.owned_elements()} owned params")
        print(json.dumps({
            "metric": "aggregated params/sec (device-resident), hierarchical "
                      + ("FedAvg (synchronous)" if sync else "FedBuff") + ", parameter-sharded",
            "value": M * C * P * world / (elapsed / args.steps), "unit": "client-params/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
            "host_issue_ms_per_step": ISSUE_S / args.steps * 1e3, "settle": SETTLE, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic (counter-based generator), rank-local slices resident in HBM",
            "config": {"workload": f"{'hier_fedavg' if sync else 'hier_fedbuff'}: {M} middles x {C} clients x {G} "
                                   f"bf16 params, parameter-sharded over {world} rank(s) "
                                   f"(flame_amd.shard.ShardedHierarchy, {plan.owned_elements()} params per rank)",
                       "middles": args.hier_mode, "middle_weights": args.hier_middles,
                       "middle_layout": args.hier_mid_layout, "arrivals": args.hier_arrivals,
                       "params_per_gpu": P, "global_params": G, "parallelism": f"param-shard{world}"},
            "roofline": {"bound": "hbm", "achieved": k_bytes / k_time / 1e9, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": k_bytes / k_time / 1e9 / PEAK_HBM_GBS, "traffic": traffic,
                         "traffic_source": traffic_source,
                         "kernel": "flame_hier_fedbuff", "kernel_ms": k_time * 1e3, "algorithmic_bytes": k_bytes,
                         "launches_per_step": lps},
            "time_attribution": attrib,
            "collective": _collective_note(plan, world, 2),
            "process_group": process_group_info(),
            "launcher": launcher(world),
            "gather_check": gc,
        }), flush=True)
    import torch.distributed as dist
    if dist.is_initialized():
        dist.destroy_process_group()
    _checked(gc)


def bench_fedbuff(args, world, rank, dev):
    """The asynchronous top aggregator (asyncfl/top_aggregator.py:54-115): aggGoal arrivals,
    each handed to FedBuff.do on its own (staleness U{0..3}), then scale_add_agg_weights
    into the model -- 64 arrivals x 25M fp32 by default, slab-resident.  --fedbuff-fuse
    off = flush the aggregate to HBM, then the separate scale_add launch."""
    from flame_amd import engine, synth
    from flame_amd.optimizers import optimizer_provider
    from flame_amd.slab import UpdateSlab
    K = args.clients or 64
    P = args.params or 25_000_000
    store = UpdateSlab({"model": torch.empty(P)}, capacity=K, device=dev)
    tmp = torch.empty(P, device=dev)
    arrivals = []
    for i in range(K):
        engine.synth_fill_(tmp, args.seed + 5, 1 + i + rank * 100_000, 0, 1e-2)
        arrivals.append(store.put({"model": tmp}))
    del tmp
    model = torch.empty(P, device=dev)
    engine.synth_fill_(model, args.seed + 5, rank * 100_000, 0, 1.0)
    stale = [int(x) % 4 for x in synth.counts(args.seed + 5, K)]
    rnd = 10
    opt = optimizer_provider.get("fedbuff", fuse_scale_add=args.fedbuff_fuse == "on")
    torch.cuda.synchronize()
    from flame_amd import _native
    br0 = _native.launch_branch_counts()

    def step():
        agg = None
        for i in range(K):     # one arrival per do(), as the role hands them over
            cache = Cache()
            cache[f"{i:05d}"] = TR(arrivals[i], 1, rnd - stale[i])
            agg = opt.do(agg, cache, total=1, version=rnd)
        opt.scale_add_agg_weights({"model": model}, agg, K)

    elapsed, events = timed(world, args.steps, args.warmup, step)
    if rank == 0:
        traffic, traffic_source = traffic_lookup(args.traffic, kernel="flame_hier_fedbuff", workload="fedbuff",
                                                 clients=K, params=P)
        kst = {nm: kernel_stats(events, nm) for nm in sorted({e[0] for e in events})}
        k_time = sum(k["avg_s"] * k["launches"] for k in kst.values()) / args.steps
        k_bytes = sum(k["bytes_per_launch"] * k["launches"] for k in kst.values()) / args.steps
        br = {k: v - br0[k] for k, v in _native.launch_branch_counts().items() if v != br0[k]}
        print(json.dumps({
            "metric": "aggregated params/sec (device-resident), async FedBuff top aggregator round",
            "value": K * P * world / (elapsed / args.steps), "unit": "client-params/s", "n_gpus": world,
            "steps": args.steps, "ms_per_step": elapsed / args.steps * 1e3, "dtype": "f32", "settle": SETTLE,
            "config": {"workload": f"fedbuff: {K} arrivals x {P} fp32 + scale_add, slab layout",
                       "fuse_scale_add": args.fedbuff_fuse},
            "roofline": {"bound": "hbm", "achieved": k_bytes / k_time / 1e9, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": k_bytes / k_time / 1e9 / PEAK_HBM_GBS, "kernel_ms_per_step": k_time * 1e3,
                         "algorithmic_bytes_per_step": k_bytes, "traffic": traffic, "traffic_source": traffic_source,
                         "bytes_per_client_param": k_bytes / (K * P * 4)},
            "kernels": kst, "launch_branches": br,
        }), flush=True)


def bench_hier(args, world, rank, dev):
    """Config 5 on one GPU's parameter shard: 64 middle aggregators x 64 clients (bf16,
    staleness U{0..3}, aggGoal 64 both levels): per middle FedBuff.do per arrival +
    fused scale_add/delta, then the top FedBuff over the 64 middle deltas + scale_add.
    Arrival batching (DeferredAggregate) turns each middle's 64 arrivals into one launch."""
    from flame_amd import engine, synth
    from flame_amd.optimizers import optimizer_provider
    from flame_amd.optimizer.fedbuff import scale_add_many
    M = 64
    C = (args.clients or 4096) // M
    P = args.params or 125_000_000 // 8
    dt = torch.bfloat16
    if world > 1 or args.force_shard:
        return bench_hier_sharded(args, world, rank, dev, M, C, P)
    from flame_amd.slab import UpdateSlab
    store = UpdateSlab({"model": torch.empty(P, dtype=dt)}, capacity=M * C, device=dev)
    tmp = torch.empty(P, dtype=dt, device=dev)
    client_w = []
    for i in range(M * C):
        engine.synth_fill_(tmp, args.seed + 4, 1 + i + rank * 100_000, 0, 1e-2)
        client_w.append(store.put({"model": tmp}))
    del tmp
    gw = torch.empty(P, dtype=dt, device=dev)
    engine.synth_fill_(gw, args.seed + 4, rank * 100_000, 0, 1.0)
    mids = [gw.clone() for _ in range(M)]
    # fused / sync modes: the middles' own weights as the slots of one tiled store (a chunk's
    # middles form one contiguous block, flame_hier_segment.mid_tile_stride) or one tensor each
    if args.hier_mid_layout == "tiled" and args.hier_mode in ("fused", "sync"):
        mid_store = UpdateSlab({"model": torch.empty(P, dtype=dt)}, capacity=M, device=dev)
        mid_w = [mid_store.put({"model": gw}) for _ in range(M)]
    else:
        mid_w = [{"model": mids[m]} for m in range(M)]
    gw_fetched = gw.clone()   # --hier-middles fetched: the model every middle fetched from the top
    stale = [int(x) % 4 for x in synth.counts(args.seed + 4, M * C)]
    rnd = 10
    mid_opts = [optimizer_provider.get("fedbuff") for _ in range(M)]
    top_opt = optimizer_provider.get("fedbuff")
    middle_arrivals = _middle_arrivals(args, M, C, client_w, stale, rnd)
    torch.cuda.synchronize()

    def step_group():
        # the middles of this node queue their arrivals, then ONE launch reduces all of
        # them (per-middle staleness rates, FLAME_AGG_SEG_RATES) and ONE launch does every
        # middle's scale_add + delta; the top FedBuff then takes the 64 deltas in one launch
        aggs = [None] * M
        for m in range(M):
            opt = mid_opts[m]
            for t in range(C):
                i = m * C + t
                cache = Cache()
                cache[f"{i:05d}"] = TR(client_w[i], 1, rnd - stale[i])
                aggs[m] = opt.do(aggs[m], cache, total=1, version=rnd)
        res = scale_add_many([({"model": mids[m]}, aggs[m]) for m in range(M)], C, with_delta=True)
        top_agg = None
        for m in range(M):
            cache = Cache()
            cache[f"mid{m:03d}"] = TR(res[m][1], C, rnd - (m % 2))
            top_agg = top_opt.do(top_agg, cache, total=C, version=rnd)
        top_opt.scale_add_agg_weights({"model": gw}, top_agg, M)

    def step_serial():
        top_agg = None
        deltas = []
        for m in range(M):
            agg = None
            opt = mid_opts[m]
            for t in range(C):
                i = m * C + t
                cache = Cache()
                cache[f"{i:05d}"] = TR(client_w[i], 1, rnd - stale[i])
                agg = opt.do(agg, cache, total=1, version=rnd)
            _, delta = opt.scale_add_agg_weights_with_delta({"model": mids[m]}, agg, C)
            deltas.append(delta)
            cache = Cache()
            cache[f"mid{m:03d}"] = TR(delta, C, rnd - (m % 2))
            top_agg = top_opt.do(top_agg, cache, total=C, version=rnd)
        top_opt.scale_add_agg_weights({"model": gw}, top_agg, M)

    from flame_amd.optimizer.fedbuff import hierarchy_round

    def step_fused():
        # every middle's arrivals queue (DeferredAggregate); ONE launch then reduces each
        # middle, applies its scale_add, feeds its delta to the top FedBuff and applies the
        # top's scale_add -- the middle aggregates and deltas stay in registers
        aggs = middle_arrivals(mid_opts)
        fetched = args.hier_middles == "fetched"
        hierarchy_round([({"model": gw_fetched} if fetched else mid_w[m], aggs[m], C, rnd - (m % 2))
                         for m in range(M)], None, version=rnd, top_weights={"model": gw}, top_goal=M,
                        update_middle_weights=not fetched)

    from flame_amd.optimizer.sync_hierarchy import sync_hierarchy_round
    counts = [int(c) for c in synth.counts(args.seed + 4, M * C)]

    def sync_caches():
        specs = []
        for m in range(M):
            cache = Cache()
            for t in range(C):
                i = m * C + t
                cache[f"{i:05d}"] = TR(client_w[i], counts[i])
            specs.append((mid_w[m], cache, sum(counts[m * C:(m + 1) * C])))
        return specs

    # the middles' caches fill as updates arrive, before the aggregation starts
    pre = [sync_caches() for _ in range(args.warmup + args.steps)] if args.hier_mode.startswith("sync") else []

    def step_sync():
        # synchronous hierarchy (syncfl middles -> syncfl top): every middle's FedAvg,
        # its delta and the top's FedAvg over the deltas in ONE launch (FLAME_HIER_SYNC)
        sync_hierarchy_round(pre.pop(), {"model": gw})

    fedavg_opt = optimizer_provider.get("fedavg")

    def step_sync_serial():
        # the same round as the roles issue it: FedAvg.do per middle, delta, FedAvg.do at the top
        top_cache = Cache()
        totals = 0
        for m, (w, cache, total) in enumerate(pre.pop()):
            new = fedavg_opt.do({"model": w["model"].clone()}, cache, total=total)
            top_cache[f"mid{m:03d}"] = TR({"model": new["model"] - w["model"]}, total)
            mids[m].copy_(new["model"])
            totals += total
        fedavg_opt.do({"model": gw}, top_cache, total=totals)

    step = {"fused": step_fused, "group": step_group, "serial": step_serial, "sync": step_sync,
            "sync_serial": step_sync_serial}[args.hier_mode]
    elapsed, events = timed(world, args.steps, args.warmup, step)
    ceiling, probes = None, {}
    if rank == 0 and world == 1:
        # the same-process read ceiling over the slab, with the kernel's own per-workgroup region
        # (every arrival's tile of one chunk: M x C x 4 KiB) beside the fastest (1 MiB) one
        ceiling, probes = read_ceiling(store.storage[dt], regions=(M * C * 4096,))
    cpu = None
    if rank == 0 and world == 1 and args.cpu_clients > 0 and not args.hier_mode.startswith("sync"):
        cpu = cpu_baseline_hier([store.read(i, "model").cpu() for i in range(C)], P, stale[:C], rnd,
                                args.cpu_rounds)
    # the roofline line prices the step's dominant kernel; every kernel the step ran is listed
    first = {"fused": "flame_hier_fedbuff", "sync": "flame_hier_fedbuff"}.get(args.hier_mode, "flame_agg_reduce")
    seen = sorted({e[0] for e in events}, key=lambda nm: (nm != first, nm))
    names = tuple(seen) if seen and seen[0] == first else (first,)
    kst = {nm: kernel_stats(events, nm) for nm in seen}
    red = kst.get(names[0]) or next(iter(kst.values()))
    traffic, traffic_source = None, None
    if rank == 0 and args.hier_mode == "fused":
        traffic, traffic_source = traffic_lookup(args.traffic, kernel=names[0], clients=M * C, params=P,
                                                 workload="hier_fedbuff" if args.hier_middles == "own"
                                                 else f"hier_fedbuff_{args.hier_middles}")
    if rank == 0:
        per_step_kernel = sum(k["avg_s"] * k["launches"] for k in kst.values()) / args.steps
        sync = args.hier_mode.startswith("sync")
        print(json.dumps({
            "metric": ("aggregated params/sec (device-resident), hierarchical "
                       + ("FedAvg (synchronous) shard" if sync else "FedBuff shard")),
            "value": M * C * P * world / (elapsed / args.steps), "unit": "client-params/s",
            "n_gpus": world, "steps": args.steps, "ms_per_step": elapsed / args.steps * 1e3,
            "host_issue_ms_per_step": ISSUE_S / args.steps * 1e3, "settle": SETTLE,
            "dtype": "bf16", "config": {"workload": f"{'hier_fedavg' if sync else 'hier_fedbuff'}: {M} middles x {C} "
                                                    f"clients x {P} bf16 per GPU",
                                        "middles": args.hier_mode, "middle_weights": args.hier_middles,
                                        "arrivals": args.hier_arrivals},
            "roofline": {"bound": "hbm", "achieved": red["achieved_GBps"], "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": red["achieved_GBps"] / PEAK_HBM_GBS, "traffic": traffic, "traffic_source": traffic_source,
                         "kernel": names[0], "kernel_ms": red["avg_s"] * 1e3,
                         "algorithmic_bytes": red["bytes_per_launch"],
                         "measured_read_ceiling_GBps": ceiling, "read_probes_GBps": probes,
                         "frac_of_measured_ceiling": red["achieved_GBps"] / ceiling if ceiling else None,
                         # against the kernel's own region read at its own residency (2 per CU, 6 loads per lane)
                         "frac_of_own_region_probe": (red["achieved_GBps"] / probes[own] if (
                             own := f"region_{(M * C * 4096) >> 20}MiB_2perCU_6ld") in probes else None)},
            "kernels": {**kst, "kernel_ms_per_step": per_step_kernel * 1e3,
                        "kernel_client_params_per_s": M * C * P / per_step_kernel},
            "cpu_baseline": cpu,
        }), flush=True)


def pcie_probe(dev, world, nbytes=256 << 20, reps=5):
    """Same-process pinned host <-> HBM copy rates, every rank at once (after a barrier): the
    PCIe ceiling each rank's link gives this process (the e2e line's roofline peak).  Ranks that
    share a GPU (the gloo rehearsal) share its link, so their aggregate is one link's."""
    host = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    host.fill_(1)
    d = torch.empty(nbytes, dtype=torch.uint8, device=dev)

    def rate(fn):
        ts = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) / 1e3)
        return nbytes / statistics.median(ts) / 1e9
    barrier(world)
    h2d = rate(lambda: d.copy_(host, non_blocking=True))
    barrier(world)
    d2h = rate(lambda: host.copy_(d, non_blocking=True))
    mine = [h2d, d2h]
    allr = gather_objects(world, mine)
    del host, d
    return {"h2d_GBps_by_rank": [round(a[0], 2) for a in allr], "d2h_GBps_by_rank": [round(a[1], 2) for a in allr],
            "h2d_aggregate_GBps": round(sum(a[0] for a in allr), 2),
            "probe": f"{nbytes >> 20} MiB pinned host <-> HBM copy per rank, all ranks at once, median of {reps}"}


def gather_objects(world, obj):
    """[obj of rank 0, ..., obj of rank world-1] (just [obj] without a process group)."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return [obj]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj)
    return out


def e2e_reference_sample(seg_names, sizes, counts, total, G, dev, budget_s=10.0, max_clients=8):
    """The reference's receive path over the same shm segments, on a bounded sample of clients
    (rank 0, untimed by the step clock): backend/shm.py:386-391 copies the message out of the
    segment, channel.py:321-325 runs cloudpickle.loads on the copy; then
    * cpu: FedAvg's op sequence on the host (fedavg.py:84-104, oracle/torch_cpu.py) -- the
      line's cpu_baseline;
    * gpu (shm_reference): weights_to_model_device (common/util.py:198-208) + the same torch
      ops on the device."""
    import cloudpickle
    from multiprocessing import shared_memory
    from oracle import torch_cpu
    res = {}
    cores, env = host_cores()
    prev = torch.get_num_threads()
    torch.set_num_threads(cores)
    try:
        for where in ("cpu", "gpu"):
            agg = {"model": torch.zeros(G, dtype=torch.float32, device="cpu" if where == "cpu" else dev)}
            t_all, k = 0.0, 0
            for i, (nm, sz) in enumerate(zip(seg_names, sizes)):
                t0 = time.perf_counter()
                seg = shared_memory.SharedMemory(nm)
                try:
                    data = bytes(seg.buf[:sz])
                finally:
                    seg.close()
                msg = cloudpickle.loads(data)
                del data
                if where == "cpu":
                    torch_cpu.fedavg_round(agg, [msg["weights"]], [int(msg["dataset_size"])], total)
                else:
                    w = {kk: v.to(dev) for kk, v in msg["weights"].items()}
                    rate = float(np.float32(int(msg["dataset_size"]) / total))
                    agg["model"] += (w["model"] * rate).to(w["model"].dtype)
                    torch.cuda.synchronize()
                t_all += time.perf_counter() - t0
                k += 1
                del msg
                if k >= max_clients or t_all >= budget_s:
                    break
            res[where] = {"clients": k, "s": round(t_all, 3), "value": k * G / t_all,
                          "host_read_GBps": k * G * 4 / t_all / 1e9}
    finally:
        torch.set_num_threads(prev)
    res["host"] = env
    return res


def bench_e2e_shm_sharded(args, world, rank, dev, n, P):
    """End to end at N GPUs: updates sit in per-sender POSIX shared-memory
    segments, as the LIFL SHM backend delivers them (backend/shm.py:393-403); every rank opens
    and hipHostRegisters the same segments once (flame_amd.ingest.ShmReceiver), decodes each
    message in place and DMAs only ITS ranges of the update into its rank-local slab
    (DeviceUpdateCache(shard=plan), its own PCIe link); ShardedOptimizer(FedAvg).do reduces the
    owned ranges wave by wave with the in-place all-gathers behind each wave, so every rank ends
    with the whole model (syncfl/top_aggregator.py:161-176); rank 0 then encodes the model
    message into a pinned egress buffer (flame_amd.egress.MessageEncoder: one D2H straight into
    the payload, syncfl/top_aggregator.py:184-215).  The step runs from "payloads in shared
    memory" to "model message in host memory".  Weak scaling: the model has P x world params."""
    import cloudpickle
    from multiprocessing import shared_memory
    from flame_amd import engine, ingest, shard, synth
    from flame_amd.egress import MessageEncoder
    from flame_amd.ingest import DeviceUpdateCache
    from flame_amd.optimizers import optimizer_provider
    n = min(n, 64)
    G = P * world
    counts = synth.counts(args.seed, n)
    total = int(counts.sum())
    gathered = args.e2e_egress == "gathered"
    sopt = shard.ShardedOptimizer(optimizer_provider.get("fedavg"), device=dev, fracs=_fracs(args, shard),
                                  gather=gathered)
    sopt.set_layout({"model": torch.empty(G, dtype=torch.float32, device="meta")})
    plan = sopt.plan
    tag = f"flamee2e{os.environ.get('MASTER_PORT', os.getpid())}"
    names = [f"{tag}_t{i}-agg" for i in range(n)]
    # the senders: rank r writes the messages of trainers r, r + world, ... (cloudpickle of
    # {weights, dataset_size}, channel.py:203-218), each into its own segment
    mine, my_sizes = [], {}
    tmp = torch.empty(G, dtype=torch.float32, device=dev)
    try:
        for i in range(rank, n, world):
            engine.synth_fill_(tmp, args.seed, 1 + i, 0, 1e-2)
            b = cloudpickle.dumps({"weights": {"model": tmp.cpu()}, "dataset_size": int(counts[i])})
            seg = shared_memory.SharedMemory(name=names[i], create=True, size=len(b))
            seg.buf[:len(b)] = b
            mine.append(seg)
            my_sizes[i] = len(b)
            del b
        del tmp
        print(f"bench.py e2e: rank {rank}: {len(mine)} trainer messages written to shared memory", file=sys.stderr,
              flush=True)
        sizes = {}
        for d in gather_objects(world, my_sizes):
            sizes.update(d)
        sizes = [sizes[i] for i in range(n)]
        barrier(world)
        _e2e_shm_sharded_run(args, world, rank, dev, n, P, G, counts, total, sopt, plan, tag, names, sizes)
    finally:
        barrier(world)
        for seg in mine:
            seg.close()
            seg.unlink()
    import torch.distributed as dist
    if dist.is_initialized():
        dist.destroy_process_group()


def _e2e_shm_sharded_run(args, world, rank, dev, n, P, G, counts, total, sopt, plan, tag, names, sizes):
    from flame_amd import engine, ingest, shard
    from flame_amd.egress import MessageEncoder
    from flame_amd.ingest import DeviceUpdateCache
    rx = ingest.ShmReceiver("agg", register=True, untrack=True)
    scache = DeviceUpdateCache(device=dev, placement="slab", capacity=n, shard=plan)
    model = torch.empty(G, dtype=torch.float32, device=dev)
    engine.synth_fill_(model, args.seed, 0, 0, 1.0)
    weights = {"model": model}
    gathered = args.e2e_egress == "gathered"
    if gathered:
        enc = MessageEncoder(ring=1) if rank == 0 else None
    else:
        from flame_amd.egress import ShardedEgress
        enc = ShardedEgress(plan, f"{tag}_egress")
    keys = [f"{i:05d}" for i in range(n)]
    phases, out = [], {}
    rounds = [0]

    def step():
        rounds[0] += 1
        e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        t0 = time.perf_counter()
        e[0].record()
        for i in range(n):          # the receive loop: decode in place, this rank's ranges -> its slab
            msg = rx.loads(f"{tag}_t{i}", sizes[i])
            scache[keys[i]] = TR(msg["weights"], msg["dataset_size"])
            del msg
        t1 = time.perf_counter()
        e[1].record()
        sopt.do(weights, scache, total=total, num_trainers=n)
        e[2].record()
        # the message every trainer gets: one encode; gathered: rank 0 D2Hs the whole model into it,
        # sharded: every rank D2Hs its ranges into the one shared payload (rank 0 receives it)
        if enc is not None:
            p = enc.encode({"weights": weights, "round": rounds[0]})
            if rank == 0:
                out["payload"] = p
        e[3].record()
        phases.append((t1 - t0, e))

    global SETTLE
    if SETTLE is None:       # PCIe-bound: no HBM settle (its 8 GB probe buffer per rank buys nothing here)
        SETTLE = {"skipped": "end-to-end line: PCIe-bound, see roofline.probe"}
    try:
        shard.GATHER_TIMING = None
        for _ in range(args.warmup):
            step()
        phases.clear()
        print(f"bench.py e2e: rank {rank}: warm-up done", file=sys.stderr, flush=True)
        shard.GATHER_TIMING = []
        elapsed, events = timed(world, args.steps, 0, step)
        gt, shard.GATHER_TIMING = shard.GATHER_TIMING, None
        torch.cuda.synchronize()
        ph = {"ingest_host_ms": statistics.mean(p[0] for p in phases) * 1e3,
              "ingest_ms": statistics.mean(p[1][0].elapsed_time(p[1][1]) for p in phases),
              "reduce_gather_ms": statistics.mean(p[1][1].elapsed_time(p[1][2]) for p in phases),
              "egress_ms": statistics.mean(p[1][2].elapsed_time(p[1][3]) for p in phases)}
        ks = kernel_stats(events, "flame_agg_reduce")
        k_ms = ks["avg_s"] * ks["launches"] / args.steps * 1e3 if ks else None
        attrib = time_attribution(world, k_ms, elapsed / args.steps * 1e3, gt)
        per_rank = gather_objects(world, ph)
        # untimed self-checks: gathered -- every rank holds the same model == the host restatement on
        # sampled elements; both -- rank 0's egress payload decodes (the trainers' cloudpickle.loads)
        # to a model whose every rank's ranges equal that rank's device copy (digests) and whose
        # sampled elements equal the host restatement, bitwise
        idx = sample_indices(plan, "model", seed=args.seed)
        expected = host_fedavg_rounds(args.seed, counts, idx, rounds[0])
        gc = verify_sharded(model, idx, expected) if gathered else {}
        gc["rounds_checked"] = rounds[0]
        ec = egress_check(plan, world, rank, model, out.get("payload"), idx, expected)
        gc.update(ec)
        if not gathered:      # (for _checked) no rank holds the whole model: the payload is the check
            gc["ranks_agree"] = ec["egress_range_mismatches"] == 0
            gc["sample_mismatches_per_rank"] = [ec["egress_sample_mismatches"]] + [0] * (world - 1)
            gc["sample_parity"] = "bitwise" if ec["egress_payload_bitwise"] else "MISMATCH"
        elif not ec["egress_payload_bitwise"]:
            gc["ranks_agree"] = False
        probe = pcie_probe(dev, world)
        ref = None
        if rank == 0 and args.cpu_clients > 0:
            ref = e2e_reference_sample(names, sizes, counts, total, G, dev)
        if rank == 0:
            ms = elapsed / args.steps * 1e3
            h2d = n * G * 4          # every update's bytes cross PCIe once (each rank its ranges)
            d2h = G * 4              # the model, once, into the egress payload
            achieved = (h2d + d2h) / (ms / 1e3) / 1e9
            peak = probe["h2d_aggregate_GBps"]
            line = {
                "metric": "aggregated params/sec, END-TO-END (LIFL shm payloads -> model message in host memory)",
                "mode": "shm (sharded ingest)", "value": n * G / (ms / 1e3), "unit": "client-params/s",
                "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms,
                "higher_is_better": True, "scaling": "weak", "dtype": "f32", "settle": SETTLE,
                "data": "synthetic (counter-based generator) cloudpickled into POSIX shm segments, one per trainer",
                "config": {"workload": f"e2e shm: {n} trainers x {G} fp32 params ({P} per GPU), parameter-sharded "
                                       f"ingest over {world} rank(s), "
                                       + ("in-place all-gathers, rank-0 egress encode" if gathered else
                                          "no all-gather, every rank's ranges D2H into one shared egress payload"),
                           "egress": args.e2e_egress,
                           "clients": n, "params_per_gpu": P, "global_params": G,
                           "parallelism": f"param-shard{world}"},
                "host_read_GBps": h2d / (ms / 1e3) / 1e9,
                "roofline": {"bound": "pcie", "achieved": achieved, "peak": peak, "unit": "GB/s",
                             "frac": achieved / peak if peak else None,
                             "spec_GBps": PCIE_SPEC_GBS * world, "frac_of_spec": achieved / (PCIE_SPEC_GBS * world),
                             "bytes_per_step": {"h2d": h2d, "d2h": d2h},
                             "per_link_achieved_GBps": h2d / world / (ms / 1e3) / 1e9,
                             "per_link_peak_GBps": probe["h2d_GBps_by_rank"], **{"probe": probe}},
                "phases_ms_by_rank": per_rank,
                "time_attribution": attrib,
                "collective": _collective_note(plan, world, 4),
                "process_group": process_group_info(), "launcher": launcher(world),
                "gather_check": gc,
                "shm_reference": None if ref is None else {
                    **ref["gpu"], "unit": "client-params/s",
                    "path": "bytes(segment[:size]) (backend/shm.py:386-391) + cloudpickle.loads (channel.py:321-325) "
                            "+ .to(device) (common/util.py:198-208) + the reference's torch ops on the device, per "
                            "trainer, rank 0 only, bounded sample"},
                "cpu_baseline": None if ref is None else {
                    "value": ref["cpu"]["value"], "unit": "client-params/s", "cores": ref["host"]["threads_used"],
                    "kind": "port", "host": ref["host"],
                    "sample": f"{ref['cpu']['clients']} trainers of the same segments: shm copy + cloudpickle.loads + "
                              f"FedAvg's op sequence on the host (oracle/torch_cpu.py), {ref['cpu']['s']} s"},
            }
            print(json.dumps(line), flush=True)
    finally:
        shard.GATHER_TIMING = None
        rx.close()
        if enc is not None and hasattr(enc, "close"):
            enc.close()
    _checked(gc)


def egress_check(plan, world, rank, model, payload, idx, expected):
    """The egress payload against the device model and the host restatement (every rank gets the
    verdict): rank 0 decodes it with cloudpickle.loads; each rank's digests of its owned ranges
    (and rank 0's of the tails) must match the same ranges of the payload, and the sampled
    elements must equal the host restatement bitwise."""
    import hashlib
    flat = model.detach().reshape(-1)

    def dig(t):
        return hashlib.blake2b(t.contiguous().view(torch.uint8).cpu().numpy(), digest_size=16).hexdigest()
    mine = [(s.lo, s.hi, dig(flat[s.lo:s.hi])) for s in plan.subs if s.hi > s.lo and (not s.tail or rank == 0)]
    allr = gather_objects(world, mine)
    res = None
    if rank == 0:
        import cloudpickle
        got = cloudpickle.loads(bytes(payload))["weights"]["model"].reshape(-1)
        bad_ranges = sum(1 for r in allr for lo, hi, d in r if dig(got[lo:hi]) != d)
        gb = got[torch.as_tensor(idx)].numpy().view(np.uint32)
        eb = np.asarray(expected, dtype=np.float32).view(np.uint32)
        res = {"egress_payload_bytes": len(payload), "egress_ranges_checked": sum(len(r) for r in allr),
               "egress_range_mismatches": bad_ranges, "egress_sample_mismatches": int(np.count_nonzero(gb != eb))}
        res["egress_payload_bitwise"] = bad_ranges == 0 and res["egress_sample_mismatches"] == 0
    return gather_objects(world, res)[0]


def time_attribution(world, k_ms, ms_per_step, gather_timing):
    """Where an N>1 step's time went, from every rank: its kernel ms per step,
    the step time not covered by the slowest rank's kernels (exposed collective + host time), and
    per wave the in-place all-gather's span on the launch stream (shard.GATHER_TIMING: from the
    wave's issue behind its kernels to its work.wait(); exact for the last wave, an upper bound
    for the ones hidden behind later waves) with the bytes this rank received."""
    waves = collections.defaultdict(list)
    for w, recv, t0, t1 in gather_timing or []:
        dt = t0.elapsed_time(t1) if hasattr(t0, "elapsed_time") else (t1 - t0) * 1e3
        waves[w].append((dt, recv))
    mine = {"kernel_ms": k_ms,
            "waves": {int(w): {"span_ms": statistics.mean(d for d, _ in v), "bytes": v[0][1], "calls": len(v)}
                      for w, v in sorted(waves.items())}}
    allr = gather_objects(world, mine)
    ks = [a["kernel_ms"] for a in allr if a["kernel_ms"] is not None]
    out = {"kernel_ms_by_rank": [a["kernel_ms"] for a in allr],
           "kernel_ms_max": max(ks) if ks else None, "kernel_ms_min": min(ks) if ks else None,
           "exposed_collective_ms": (ms_per_step - max(ks)) if ks else None, "allgather": []}
    for w in sorted({w for a in allr for w in a["waves"]}):
        spans = [a["waves"][w]["span_ms"] if w in a["waves"] else None for a in allr]
        nbytes = allr[0]["waves"].get(w, {}).get("bytes", 0)
        sp = [s for s in spans if s is not None]
        out["allgather"].append({"wave": w, "bytes_received_per_rank": nbytes, "span_ms_by_rank": spans,
                                 "GBps": nbytes / (max(sp) / 1e3) / 1e9 if sp and max(sp) > 0 else None})
    if out["allgather"]:
        last = out["allgather"][-1]
        out["last_wave_exposed_gather_ms"] = max(s for s in last["span_ms_by_rank"] if s is not None)
    return out


def bench_e2e(args, n, P, dev):
    """Host-resident updates -> FedAvg on the GPU -> global model back in host memory.

    zerocopy: the reduction kernel reads the pinned host updates directly over PCIe
              (no staging copy, no HBM footprint for updates);
    copy:     pinned host -> HBM on a copy stream, double-buffered batches overlapped
              with the reduction of the previous batch;
    pageable: the reference convention (weights_to_model_device: per-tensor .to(device)
              from pageable memory), then one FedAvg;
    shard:    the parameter-sharded ingest + round: every arrival goes into
              DeviceUpdateCache(shard=plan) (this rank's ranges, strided H2D on its side
              stream, into the rank-local slab), then ShardedOptimizer(FedAvg).do (waves +
              in-place gathers; at world 1 the gathers are no-ops);
    eager:    the eager top aggregator (eager_syncfl/top_aggregator.py:36-90): every arrival
              goes into a DeviceUpdateCache (H2D on its side stream) and FedAvg.do runs
              per arrival with the running total, so the reduction trails the transfers;
    wire*:    starts from the channel's serialized payloads (cloudpickle of
              {weights, dataset_size}, channel.py:203-218): wire = flame_amd.ingest.decode
              (zero-copy views into the payload bytes) + H2D; wire_pinned = payloads sit in
              pinned receive buffers, decode gives device-addressable views the kernel streams
              directly; wire_reference = cloudpickle.loads + .to(device) (the reference ingest);
    shm*:     payloads sit in per-sender POSIX shared-memory segments (the LIFL SHM backend,
              backend/shm.py:386-403): shm = flame_amd.ingest.ShmReceiver (segments registered
              once, decoded in place, the kernel streams the views); shm_reference = the
              backend's bytes(buf[:size]) copy + cloudpickle.loads + .to(device)."""
    from flame_amd import engine, synth
    from flame_amd.optimizers import optimizer_provider
    n = min(n, 64)
    batch = 8
    mode = args.e2e_mode
    host = torch.empty((n, P), dtype=torch.float32, pin_memory=(mode in ("zerocopy", "copy", "eager", "shard")))
    tmp = torch.empty(P, dtype=torch.float32, device=dev)
    for i in range(n):
        engine.synth_fill_(tmp, args.seed, 1 + i, 0, 1e-2)
        host[i].copy_(tmp)
    base_h = torch.empty(P, dtype=torch.float32).pin_memory()
    engine.synth_fill_(tmp, args.seed, 0, 0, 1.0)
    base_h.copy_(tmp)
    counts = synth.counts(args.seed, n)
    total = int(counts.sum())
    opt = optimizer_provider.get("fedavg")
    if mode == "eager" and args.eager_defer == "on":
        opt = optimizer_provider.get("fedavg", defer=True)
    out_h = torch.empty(P, dtype=torch.float32).pin_memory()
    if mode.startswith("wire"):
        import cloudpickle
        from flame_amd import ingest
        payloads = []
        for i in range(n):
            # a trainer's update owns its storage (pickling a view would ship the whole slab)
            b = cloudpickle.dumps({"weights": {"model": host[i].clone()}, "dataset_size": int(counts[i])})
            if mode == "wire_pinned":
                pb = torch.empty(len(b), dtype=torch.uint8, pin_memory=True)
                pb.numpy()[:] = memoryview(b)
                payloads.append(pb.numpy())
            else:
                payloads.append(b)
        del host
    shm_segs = []
    if mode.startswith("shm"):
        import cloudpickle
        from multiprocessing import shared_memory
        from flame_amd import ingest
        sizes = []
        tag = f"flamebench{os.getpid()}"
        for i in range(n):
            b = cloudpickle.dumps({"weights": {"model": host[i].clone()}, "dataset_size": int(counts[i])})
            seg = shared_memory.SharedMemory(name=f"{tag}_t{i}-agg", create=True, size=len(b))
            seg.buf[:len(b)] = b
            shm_segs.append(seg)
            sizes.append(len(b))
            del b
        del host
        rx = ingest.ShmReceiver("agg", untrack=False)
    if mode == "copy":
        dslab = torch.empty((2, batch, P), dtype=torch.float32, device=dev)
        copy_stream = torch.cuda.Stream(dev)
    if mode == "eager":
        from flame_amd.ingest import DeviceUpdateCache
        ecache = DeviceUpdateCache(device=dev, placement=args.e2e_placement, capacity=n)
    if mode == "shard":
        from flame_amd import shard
        from flame_amd.ingest import DeviceUpdateCache
        sopt = shard.ShardedOptimizer(opt, device=dev)
        sopt.set_layout({"model": torch.empty(P, dtype=torch.float32, device="meta")})
        scache = DeviceUpdateCache(device=dev, placement="slab", capacity=n, shard=sopt.plan)
    torch.cuda.synchronize()

    def step():
        base = base_h.to(dev, non_blocking=True)
        if mode == "zerocopy":
            cache = Cache()
            for i in range(n):
                cache[f"{i:05d}"] = TR({"model": host[i]}, int(counts[i]))
            opt.do({"model": base}, cache, total=total)
        elif mode.startswith("wire"):
            cache = Cache()
            for i in range(n):
                if mode == "wire_reference":
                    msg = cloudpickle.loads(payloads[i])
                    w = {k: v.to(dev) for k, v in msg["weights"].items()}
                else:
                    msg = ingest.decode(payloads[i])
                    w = msg["weights"]
                cache[f"{i:05d}"] = TR(w, msg["dataset_size"])
            opt.do({"model": base}, cache, total=total)
        elif mode.startswith("shm"):
            cache = Cache()
            for i in range(n):
                if mode == "shm_reference":   # backend/shm.py:386-391 + channel.py:321-325 + util.py:198-208
                    buf = shared_memory.SharedMemory(f"{tag}_t{i}-agg")
                    data = bytes(buf.buf[:sizes[i]])
                    buf.close()
                    msg = cloudpickle.loads(data)
                    w = {k: v.to(dev) for k, v in msg["weights"].items()}
                else:
                    msg = rx.loads(f"{tag}_t{i}", sizes[i])
                    w = msg["weights"]
                cache[f"{i:05d}"] = TR(w, msg["dataset_size"])
                del msg
            opt.do({"model": base}, cache, total=total)
            del cache, w
        elif mode == "shard":
            for i in range(n):   # arrival i: this rank's ranges -> the rank-local slab (side stream)
                scache[f"{i:05d}"] = TR({"model": host[i]}, int(counts[i]))
            sopt.do({"model": base}, scache, total=total)
        elif mode == "eager":
            base_w = {"model": base}
            running = 0
            for i in range(n):   # arrival i: receive -> cache (H2D on the side stream) -> do()
                running += int(counts[i])
                ecache[f"{i:05d}"] = TR({"model": host[i]}, int(counts[i]))
                res = opt.do(base_w, ecache, total=running, num_trainers=n)
            base = res["model"]       # the role reads the returned object (a deferred round flushes)
        elif mode == "pageable":
            cache = Cache()
            for i in range(n):  # weights_to_model_device (common/util.py:198-208)
                cache[f"{i:05d}"] = TR({"model": host[i].to(dev)}, int(counts[i]))
            opt.do({"model": base}, cache, total=total)
        else:
            cur = torch.cuda.current_stream(dev)
            done = [torch.cuda.Event(), torch.cuda.Event()]
            for b0 in range(0, n, batch):
                slot = (b0 // batch) % 2
                with torch.cuda.stream(copy_stream):
                    if b0 >= 2 * batch:
                        copy_stream.wait_event(done[slot])
                    for j in range(batch):
                        dslab[slot, j].copy_(host[b0 + j], non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(copy_stream)
                cur.wait_event(ev)
                cache = Cache()
                for j in range(batch):
                    cache[f"{b0 + j:05d}"] = TR({"model": dslab[slot, j]}, int(counts[b0 + j]))
                # batch after batch with the final total == one FedAvg over all (same order, same ops)
                opt.do({"model": base}, cache, total=total)
                done[slot].record(cur)
        out_h.copy_(base, non_blocking=True)

    try:
        elapsed, events = timed(1, args.steps, args.warmup, step)
    finally:
        if shm_segs:
            rx.close()
            for seg in shm_segs:
                seg.close()
                seg.unlink()
    ks = kernel_stats(events, "flame_agg_reduce")
    probe = pcie_probe(dev, 1)
    ms = elapsed / args.steps * 1e3
    # bytes over PCIe per step: every update in (the wire modes: their payloads' tensors), the base
    # model in and the aggregated model out (out_h)
    h2d, d2h = (n + 1) * P * 4, P * 4
    achieved = (h2d + d2h) / (ms / 1e3) / 1e9
    print(json.dumps({
        "metric": "aggregated params/sec, END-TO-END (host-resident updates -> global model in host memory)",
        "mode": mode, "value": n * P / (ms / 1e3), "unit": "client-params/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms, "clients": n, "params": P, "settle": SETTLE,
        "host_read_GBps": n * P * 4 / (ms / 1e3) / 1e9,
        "kernel_ms_per_step": ks["avg_s"] * ks["launches"] / args.steps * 1e3,
        "roofline": {"bound": "pcie", "achieved": achieved, "peak": probe["h2d_aggregate_GBps"], "unit": "GB/s",
                     "frac": achieved / probe["h2d_aggregate_GBps"], "bytes_per_step": {"h2d": h2d, "d2h": d2h},
                     "spec_GBps": PCIE_SPEC_GBS, "frac_of_spec": achieved / PCIE_SPEC_GBS,
                     "note": "peak = this process's pinned-copy probe (one SDMA copy); a kernel streaming "
                             "pinned memory, or copies from a registered segment, can read a few % above it",
                     "probe": probe},
        "launcher": launcher(1),
    }), flush=True)


if __name__ == "__main__":
    try:
        main()
    except SystemExit:
        raise
    except BaseException as e:  # noqa: BLE001 - name the rank, fail non-zero (no restart)
        import traceback
        traceback.print_exc()
        print(f"bench.py: rank {os.environ.get('RANK', '0')} of {os.environ.get('WORLD_SIZE', '1')} failed: "
              f"{type(e).__name__}: {e}", file=sys.stderr, flush=True)
        sys.exit(3)
