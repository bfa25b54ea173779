#!/usr/bin/env python3
"""Per-round HBM bytes of the eager FedAvg round from the PMC passes of tools/gpu_eager_pmc.sh
(gfx950 corrections as tools/pmc_traffic.py: read = 2 * FETCH_SIZE KiB, write = WRITE_SIZE KiB)."""
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_traffic import per_dispatch  # noqa: E402

out = sys.argv[1]
P, N = 25_000_000, 64
for mode, launches in (("on", 1), ("off", 64)):
    f = per_dispatch(f"{out}/{mode}_FETCH_SIZE", "FETCH_SIZE", "agg_reduce")
    w = per_dispatch(f"{out}/{mode}_WRITE_SIZE", "WRITE_SIZE", "agg_reduce")
    steps = len(f) // launches
    rd = 2 * sum(f) * 1024 / steps
    wr = sum(w) * 1024 / (len(w) // launches)
    alg = (N + 2 * launches) * P * 4
    print(f"defer {mode}: {len(f)} dispatches ({launches}/round), HBM read {rd / 1e9:.3f} GB + write "
          f"{wr / 1e9:.3f} GB per round = {(rd + wr) / (N * P * 4):.4f} bytes per client-param byte; "
          f"algorithmic {alg / 1e9:.3f} GB ({(rd + wr) / alg:.5f} x)")
