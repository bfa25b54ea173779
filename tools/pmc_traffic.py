#!/usr/bin/env python3
"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into HBM bytes per launch.

gfx950 corrections (MI355X_MICROARCH.md §HBM): counters are in KiB;
FETCH_SIZE reports exactly HALF the bytes of a wide (16 B/lane) coalesced
streaming read, so read bytes = 2 * FETCH_SIZE * 1024; WRITE_SIZE is exact for
16-B-per-lane streaming stores.  Writes profiles/traffic.json for bench.py.

    python tools/pmc_traffic.py --fetch DIR1 --write DIR2 --kernel agg_reduce \
        --clients 1024 --params 25000000 --out profiles/traffic.json
"""
import argparse
import csv
import glob
import json
import os
import statistics


def per_dispatch(d, counter, kernel):
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if kernel not in row.get("Kernel_Name", "") or row.get("Counter_Name") != counter:
                continue
            key = row.get("Dispatch_Id") or row.get("Correlation_Id")
            vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    return list(vals.values())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--kernel", default="agg_reduce")
    ap.add_argument("--name", default="flame_agg_reduce")
    ap.add_argument("--clients", type=int, default=1024)
    ap.add_argument("--params", type=int, default=25_000_000)
    ap.add_argument("--out", default="profiles/traffic.json")
    ap.add_argument("--layout", default="slab")
    ap.add_argument("--workload", default=None,
                    help="bench.py workload the passes ran (part of the entry's key: FedAdam / FedYogi / "
                         "FedAdaGrad share a kernel name)")
    ap.add_argument("--itemsize", type=int, default=4, help="bytes per element (bf16: 2)")
    ap.add_argument("--source", default=None,
                    help="where the counters came from (committed CSVs under profiles/ + run id); bench.py "
                         "copies it into roofline.traffic_source")
    ap.add_argument("--extra-arrays", type=int, default=2,
                    help="P-sized arrays besides the N clients in the algorithmic bytes (FedAvg 2, FedOPT 8)")
    a = ap.parse_args()
    fetch = per_dispatch(a.fetch, "FETCH_SIZE", a.kernel)
    write = per_dispatch(a.write, "WRITE_SIZE", a.kernel)
    if not fetch or not write:
        raise SystemExit(f"no counter rows for {a.kernel}: fetch={len(fetch)} write={len(write)}")
    f_kb, w_kb = statistics.median(fetch), statistics.median(write)
    read_b = 2.0 * f_kb * 1024
    write_b = w_kb * 1024
    algo = (a.clients + a.extra_arrays) * a.params * a.itemsize
    res = {
        "kernel": a.name, "clients": a.clients, "params": a.params, "layout": a.layout,
        **({"workload": a.workload} if a.workload else {}),
        "fetch_size_kb_median": f_kb, "write_size_kb_median": w_kb, "dispatches": [len(fetch), len(write)],
        "hbm_read_bytes_per_launch": read_b, "hbm_write_bytes_per_launch": write_b,
        "hbm_bytes_per_launch": read_b + write_b,
        "algorithmic_bytes_per_launch": algo,
        "traffic_over_algorithmic": (read_b + write_b) / algo,
        "correction": "read = 2*FETCH_SIZE KiB (gfx950 half-count on 16B/lane streams), write = WRITE_SIZE KiB",
        "source": a.source or f"rocprofv3 --pmc FETCH_SIZE: {a.fetch}; --pmc WRITE_SIZE: {a.write}",
    }
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    # the file holds one entry per (kernel, clients, params, layout); replace ours
    try:
        doc = json.load(open(a.out))
        entries = doc["entries"] if "entries" in doc else [doc]
    except Exception:  # noqa: BLE001
        entries = []
    key = lambda e: (e.get("kernel"), e.get("clients"), e.get("params"), e.get("layout", "row"),  # noqa: E731
                     e.get("workload"))
    entries = [e for e in entries if key(e) != key(res)] + [res]
    json.dump({"entries": entries}, open(a.out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
