#!/usr/bin/env python3
"""Print the device's free / total VRAM (hipMemGetInfo) every --every seconds for --secs seconds,
to see how long a finished process's memory takes to come back (cross-process spread)."""
import argparse
import time

import torch

ap = argparse.ArgumentParser()
ap.add_argument("--secs", type=float, default=0)
ap.add_argument("--every", type=float, default=2)
a = ap.parse_args()
t0 = time.time()
while True:
    free, total = torch.cuda.mem_get_info(0)
    print(f"t={time.time() - t0:6.1f}s free {free / 1e9:7.1f} GB of {total / 1e9:7.1f} GB", flush=True)
    if time.time() - t0 >= a.secs:
        break
    time.sleep(a.every)
