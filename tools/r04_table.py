#!/usr/bin/env python3
"""Print DESIGN.md §0's shipped-build table from round 4's evidence files.

For each default path: the bench line (kernel time from HIP events, ms / step, roofline frac)
and the rocprofv3 kernel-trace summary of the SAME process (average duration of the path's
kernel), plus the PMC traffic / algorithmic ratio from profiles/traffic.json.

    python tools/r04_table.py
"""
import csv
import glob
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = os.path.join(ROOT, "profiles")

PATHS = [  # tag, label, kernel-name substring in the trace summary, traffic.json match
    ("fedavg", "C3 FedAvg 1024 x 25M fp32 (headline)", "agg_reduce_kernel", ("flame_agg_reduce", 1024, "fedavg")),
    ("fedadam", "C4 FedAdam 1024 x 25M fp32, adaptive round", "fedopt_kernel", ("flame_fedopt_reduce_adapt", 1024, "fedadam")),
    ("fedyogi", "C4 FedYogi", "fedopt_kernel", ("flame_fedopt_reduce_adapt", 1024, "fedyogi")),
    ("fedadagrad", "C4 FedAdaGrad", "fedopt_kernel", ("flame_fedopt_reduce_adapt", 1024, "fedadagrad")),
    ("hier_fedbuff", "C5 shard 64 x 64 x 15.6M bf16, own middles", "hier_fedbuff_kernel", ("flame_hier_fedbuff", 4096, "hier_fedbuff")),
    ("fedbuff", "async FedBuff top, 64 x 25M fp32 + scale_add", "hier_fedbuff_kernel", ("flame_hier_fedbuff", 64, "fedbuff")),
]


def bench_line(path):
    for ln in open(path):
        if ln.startswith("{"):
            return json.loads(ln)
    return None


def trace_avg(tag, sub):
    for f in glob.glob(os.path.join(P, f"r04prof_{tag}_kernel_stats.csv")):
        rows = [r for r in csv.DictReader(open(f)) if sub in r.get("Name", "")]
        if rows:
            r = max(rows, key=lambda r: float(r["TotalDurationNs"]))
            return float(r["AverageNs"]) / 1e6, int(r["Calls"])
    return None, None


def main():
    traffic = json.load(open(os.path.join(P, "traffic.json")))["entries"]
    print("| path | kernel (HIP events) | trace avg (same process) | ms / step | frac | frac of the process's probe ceiling | PMC / algorithmic | files |")
    print("|---|---|---|---|---|---|---|---|")
    for tag, label, sub, (kname, clients, wl) in PATHS:
        f = os.path.join(P, f"r04prof_prof_{tag}.log")
        if not os.path.exists(f):
            continue
        b = bench_line(f)
        rf = b["roofline"]
        kms = rf.get("kernel_ms") or rf.get("kernel_ms_per_step")
        avg, calls = trace_avg(tag, sub)
        tr = [e for e in traffic if e.get("kernel") == kname and e.get("clients") == clients and e.get("workload") == wl]
        ratio = tr[-1]["traffic_over_algorithmic"] if tr else None
        fc = rf.get("frac_of_measured_ceiling")
        ceil = f"{fc:.3f} ({rf['measured_read_ceiling_GBps'] / 1e3:.2f} TB/s)" if fc else "--"
        print(f"| {label} | {kms:.3f} ms | {avg:.3f} ms x {calls} |" if avg else f"| {label} | {kms:.3f} ms | -- |",
              f"{b['ms_per_step']:.3f} | {rf['frac']:.3f} | {ceil} |",
              f"{ratio:.6f} |" if ratio else "-- |",
              f"`r04prof_prof_{tag}.log`, `r04prof_{tag}_kernel_stats.csv` |")


if __name__ == "__main__":
    main()
