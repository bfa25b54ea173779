#!/usr/bin/env python3
"""Is the cross-process spread the allocation or the box's state?  In ONE process:
allocate a 102.4 GB buffer, run the same-process read probes (bench.read_ceiling) a few times,
free it (and the caching allocator's blocks), allocate again, probe again; optionally keep the
HBM busy streaming for --heat seconds between the two halves.  A slower second half after a
re-allocation points at the allocation (physical placement); a slower half after streaming
alone points at the box's state (temperature).

    python tools/state_probe.py --gb 102.4 --heat 40
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=102.4)
    ap.add_argument("--heat", type=float, default=40.0, help="seconds of streaming reads between the halves")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import bench
    dev = torch.device("cuda", 0)
    n = int(a.gb * 1e9) // 4
    out = {}

    def probe(tag, buf):
        best, res = bench.read_ceiling(buf, reps=a.reps)
        out[tag] = {"best_GBps": best, **res}
        print(tag, json.dumps({k: round(v) for k, v in out[tag].items()}), flush=True)

    buf = torch.ones(n, dtype=torch.float32, device=dev)
    probe("alloc1_cold", buf)
    t0 = time.time()
    while time.time() - t0 < a.heat:
        bench.read_ceiling(buf, reps=1)
    probe("alloc1_after_heat", buf)
    del buf
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    buf = torch.ones(n, dtype=torch.float32, device=dev)
    probe("alloc2", buf)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
