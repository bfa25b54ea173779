#!/usr/bin/env python3
"""Archive a gpu_session.py evidence collection into profiles/ and print DESIGN.md's tables.

    python tools/evidence.py --archive r06fin     # gpurun_out/r06fin_* -> profiles/r06fin_*
    python tools/evidence.py r06fin               # the tables, from profiles/

Layout written by tools/gpu_session.py: the step log gpurun_out/<tag>_<step>.log (the bench line
is its last JSON line); a rocprofv3 step's summary gpurun_out/<tag>/<step>/run_kernel_stats.csv; a
PMC step's counters gpurun_out/<tag>/<step>/run_counter_collection.csv.  PMC pairs
(pmc_<path>_FETCH_SIZE / _WRITE_SIZE) are turned into profiles/traffic.json entries by
tools/pmc_traffic.py (run separately, its --source naming the archived CSVs).
"""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = os.path.join(ROOT, "profiles")
O = os.path.join(ROOT, "gpurun_out")
KERNEL = {"fedavg": "agg_reduce_kernel", "fedadam": "fedopt_kernel", "fedyogi": "fedopt_kernel",
          "fedadagrad": "fedopt_kernel", "hier_fedbuff": "hier_fedbuff_kernel<", "fedbuff": "hier_fedbuff_kernel",
          "fedadam_eager": "fedopt_chain_kernel", "fedyogi_eager": "fedopt_chain_kernel",
          "fedadagrad_eager": "fedopt_chain_kernel", "feddyn": "feddyn_kernel", "chain_bf16": "fedopt_chain_kernel"}


def archive(t):
    n = 0
    for log in sorted(glob.glob(os.path.join(O, f"{t}_*.log"))):
        shutil.copy(log, os.path.join(P, os.path.basename(log)))
        n += 1
    for d in sorted(glob.glob(os.path.join(O, t, "*"))):
        step = os.path.basename(d)
        for name, suffix in (("run_kernel_stats.csv", "kernel_stats.csv"),
                             ("run_counter_collection.csv", "counters.csv")):
            src = os.path.join(d, name)
            if os.path.exists(src):
                shutil.copy(src, os.path.join(P, f"{t}_{step}_{suffix}"))
                n += 1
    print(f"archived {n} files as profiles/{t}_*", flush=True)


def line(path):
    rows = [json.loads(x) for x in open(path) if x.startswith("{")]
    return rows[-1] if rows else None


def stats(t, step, kernel):
    f = os.path.join(P, f"{t}_{step}_kernel_stats.csv")
    if not os.path.exists(f):
        return None
    ks = [x for x in csv.DictReader(open(f)) if kernel in x["Name"]]
    return max(ks, key=lambda x: int(x["Calls"])) if ks else None


def table(t):
    print("| path | kernel (HIP events) | trace avg (same process) | ms / step | frac | of probe ceiling | "
          "PMC / algorithmic | file |")
    print("|---|---|---|---|---|---|---|---|")
    for f in sorted(glob.glob(os.path.join(P, f"{t}_prof_*.log"))):
        step = os.path.basename(f)[len(t) + 1:-4]
        w = step[len("prof_"):]
        d = line(f)
        if d is None or "roofline" not in d:
            continue
        r = d["roofline"]
        k = r.get("kernel_ms") or r.get("kernel_ms_per_step")
        ks = stats(t, step, KERNEL.get(w, w))
        tr = f"{float(ks['AverageNs']) / 1e6:.3f} ms x {ks['Calls']}" if ks else "--"
        ratio = (r.get("traffic_source") or {}).get("traffic_over_algorithmic")
        fc = r.get("frac_of_measured_ceiling")
        print(f"| {w} | {k:.3f} ms | {tr} | {d['ms_per_step']:.3f} | {r['frac']:.3f} | "
              f"{f'{fc:.3f}' if fc else '--'} | {f'{ratio:.6f}' if ratio else '--'} | `{os.path.basename(f)}` |")
    print()
    print("| other lines | ms / step | value | roofline | file |")
    print("|---|---|---|---|---|")
    for f in sorted(glob.glob(os.path.join(P, f"{t}_*.log"))):
        step = os.path.basename(f)[len(t) + 1:-4]
        if step.startswith(("prof_", "pmc_")):
            continue
        d = line(f)
        if d is None or "ms_per_step" not in d:
            continue
        r = d.get("roofline") or {}
        print(f"| {step} ({d.get('n_gpus', 1)} GPU) | {d['ms_per_step']:.3f} | {d['value']:.4g} | "
              f"{r.get('bound')} {r.get('frac', 0):.3f} of {r.get('peak', 0):.0f} | `{os.path.basename(f)}` |")


if __name__ == "__main__":
    if sys.argv[1] == "--archive":
        archive(sys.argv[2])
        table(sys.argv[2])
    else:
        table(sys.argv[1])
