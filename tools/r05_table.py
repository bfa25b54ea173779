#!/usr/bin/env python3
"""Print DESIGN.md §0's shipped-build tables from an archived evidence collection
(tools/gpu_r05_prof.sh, copied into profiles/ by `--archive`).

    python tools/r05_table.py --archive r05fin   # gpurun_out/r05fin -> profiles/r05fin_*
    python tools/r05_table.py r05fin             # the tables, from profiles/
"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = os.path.join(ROOT, "profiles")
PROF = ["fedavg", "fedadam", "fedyogi", "fedadagrad", "hier_fedbuff", "fedbuff", "fedadam_eager", "fedyogi_eager",
        "fedadagrad_eager", "feddyn"]
PLAIN = ["c2", "fedavg_eager", "scaffold", "hier_fetched", "hier_sync"]
PMC = ["fedavg", "fedadam_eager", "hier_fedbuff"]
KERNEL = {"fedavg": "agg_reduce_kernel", "fedadam": "fedopt_kernel", "fedyogi": "fedopt_kernel",
          "fedadagrad": "fedopt_kernel", "hier_fedbuff": "hier_fedbuff_kernel<", "fedbuff": "hier_fedbuff_kernel_argmeta",
          "fedadam_eager": "fedopt_chain_kernel", "fedyogi_eager": "fedopt_chain_kernel",
          "fedadagrad_eager": "fedopt_chain_kernel", "feddyn": "feddyn_kernel"}


def archive(t):
    o = os.path.join(ROOT, "gpurun_out", t)
    for w in PROF:
        shutil.copy(os.path.join(o, f"{w}.log"), os.path.join(P, f"{t}_{w}.log"))
        shutil.copy(os.path.join(o, w, "run_kernel_stats.csv"), os.path.join(P, f"{t}_{w}_kernel_stats.csv"))
    for w in PLAIN:
        shutil.copy(os.path.join(o, f"bench_{w}.log"), os.path.join(P, f"{t}_bench_{w}.log"))
    for w in PMC:
        for c in ("FETCH_SIZE", "WRITE_SIZE"):
            shutil.copy(os.path.join(o, f"pmc_{w}_{c}", "run_counter_collection.csv"),
                        os.path.join(P, f"{t}_pmc_{w}_{c}.csv"))
    shutil.copy(os.path.join(o, "traffic.json"), os.path.join(P, "traffic.json"))


def line(path):
    return [json.loads(x) for x in open(path) if x.startswith("{")][-1]


def table(t):
    print("| path | kernel (HIP events) | trace avg (same process) | ms / step | frac | frac of probe ceiling | traffic / algorithmic |")
    print("|---|---|---|---|---|---|---|")
    for w in PROF:
        d = line(os.path.join(P, f"{t}_{w}.log"))
        r = d["roofline"]
        k = r.get("kernel_ms") or r.get("kernel_ms_per_step")
        ks = [x for x in csv.DictReader(open(os.path.join(P, f"{t}_{w}_kernel_stats.csv"))) if KERNEL[w] in x["Name"]]
        ks = max(ks, key=lambda x: int(x["Calls"]))
        src = r.get("traffic_source") or {}
        ratio = src.get("traffic_over_algorithmic")
        print(f"| {w} | {k:.3f} ms | {float(ks['AverageNs']) / 1e6:.3f} ms x {ks['Calls']} | {d['ms_per_step']:.3f} | "
              f"{r['frac']:.3f} | {r.get('frac_of_measured_ceiling') or '--'} | {ratio if ratio else '--'} |")
    print()
    print("| workload | ms / step | kernel ms / step | frac |")
    print("|---|---|---|---|")
    for w in PLAIN:
        d = line(os.path.join(P, f"{t}_bench_{w}.log"))
        r = d["roofline"]
        k = r.get("kernel_ms") or r.get("kernel_ms_per_step")
        print(f"| {w} | {d['ms_per_step']:.3f} | {k if k is None else round(k, 3)} | {r['frac']:.3f} "
              f"({r.get('frac_of_measured_ceiling')}) |")


if __name__ == "__main__":
    if sys.argv[1] == "--archive":
        archive(sys.argv[2])
        table(sys.argv[2])
    else:
        table(sys.argv[1])
