#!/usr/bin/env python3
"""Durations of, and idle gaps between, consecutive launches of one kernel in a rocprofv3
--kernel-trace CSV (the steady-state steps of a bench).  python tools/kernel_gaps.py DIR NAME"""
import csv
import glob
import os
import statistics
import sys


def main():
    d, name = sys.argv[1], sys.argv[2]
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    ks = [(s, e) for s, e, n in rows if name in n]
    if len(ks) < 3:
        raise SystemExit(f"{len(ks)} launches of {name}")
    ks = ks[len(ks) // 4:]                                   # steady state
    dur = [(e - s) / 1e3 for s, e in ks]
    gaps = [(ks[i + 1][0] - ks[i][1]) / 1e3 for i in range(len(ks) - 1)]
    between = {}
    for i in range(len(ks) - 1):                             # what else ran in each gap
        for s, e, n in rows:
            if ks[i][1] <= s < ks[i + 1][0] and name not in n:
                between[n[:60]] = between.get(n[:60], 0) + 1
    print(f"{name}: {len(ks)} launches  duration median {statistics.median(dur):.2f} us  "
          f"gap median {statistics.median(gaps):.2f} us  p10 {sorted(gaps)[len(gaps) // 10]:.2f}  "
          f"p90 {sorted(gaps)[9 * len(gaps) // 10]:.2f}")
    for n, c in sorted(between.items(), key=lambda x: -x[1])[:10]:
        print(f"  in gaps: {c:6d} x {n}")


if __name__ == "__main__":
    main()
