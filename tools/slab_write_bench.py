"""Slab insert timing (VERDICT r02 "next" #3): one 25M-param fp32 update (100 MB) into a tiled
UpdateSlab slot, per source kind and method, HIP events on the insert stream, median of R.

    python tools/slab_write_bench.py [--params 25000000] [--capacity 16] [--reps 20]

Methods: `kernel` = flame_slab_write (one launch), `torch` = the round-2 path (torch copy_ into
the strided slot view), `2d` = flame_slab_write_2d (hipMemcpy2DAsync), `mapped` = the kernel
reading a pinned host source through its device mapping (PCIe)."""
import argparse
import os
import statistics
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flame_amd import _native as N  # noqa: E402
from flame_amd import engine  # noqa: E402
from flame_amd.slab import UpdateSlab  # noqa: E402


def torch_write(slab, slot, w):
    for k in slab.keys:
        dt, shape, n, tile0, tiles = slab.meta[k]
        src = w[k].reshape(-1)
        view = slab.slot_view(slot, k)
        T = view.shape[1]
        full = n // T
        if full:
            view[:full].copy_(src[:full * T].view(full, T), non_blocking=True)
        if n % T:
            view[full, :n % T].copy_(src[full * T:], non_blocking=True)


def raw_write(slab, slot, w, fn, mapped=False):
    wt = slab._write_table()
    rows = []
    for i, k in enumerate(slab.keys):
        p = w[k].data_ptr()
        if mapped:
            p = engine.host_device_pointer(p)
        rows.append((p, int(wt[i, 0]) + slot * N.FLAME_TILE_BYTES, int(wt[i, 1]), int(wt[i, 2])))
    tab = np.asarray(rows, dtype=np.uint64).view(np.int64)
    N.check(getattr(N.lib(), fn)(tab.ctypes.data, len(rows), torch.cuda.current_stream().cuda_stream))


def timeit(fn, reps):
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    return statistics.median(ts), min(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--params", type=int, default=25_000_000)
    ap.add_argument("--capacity", type=int, default=64)   # > 2 GiB: torch splits its strided copy
    ap.add_argument("--cases", default="all", choices=["all", "device"])
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    tmpl = {"model": torch.empty(a.params)}
    slab = UpdateSlab(tmpl, a.capacity, dev)
    nbytes = a.params * 4
    srcd = {"model": torch.randn(a.params, device=dev)}
    srch = {"model": srcd["model"].cpu().pin_memory()}
    srcp = {"model": srcd["model"].cpu()}
    print(f"insert of {nbytes / 1e6:.0f} MB into a {a.capacity}-slot slab ({torch.cuda.get_device_name(0)})")
    cases = [
        ("device  kernel (flame_slab_write, UpdateSlab.write)", lambda: slab.write(3, srcd), 2 * nbytes),
        ("device  torch copy_ (round 2)", lambda: torch_write(slab, 4, srcd), 2 * nbytes),
        ("device  2d (hipMemcpy2DAsync D2D)", lambda: raw_write(slab, 5, srcd, "flame_slab_write_2d"), 2 * nbytes),
        ("pinned  2d (flame_slab_write_2d, UpdateSlab.write)", lambda: slab.write(6, srch), nbytes),
        ("pinned  torch copy_ (round 2)", lambda: torch_write(slab, 7, srch), nbytes),
        ("pinned  kernel over the host mapping", lambda: raw_write(slab, 8, srch, "flame_slab_write", True), nbytes),
        ("pageable 2d (UpdateSlab.write)", lambda: slab.write(9, srcp), nbytes),
        ("pageable torch copy_ (round 2)", lambda: torch_write(slab, 10, srcp), nbytes),
    ]
    if a.cases == "device":
        cases = cases[:3]
    for name, fn, traffic in cases:
        fn()
        torch.cuda.synchronize()
        med, mn = timeit(fn, a.reps)
        print(f"{name:55s} median {med * 1e3:9.1f} us  min {mn * 1e3:9.1f} us  {traffic / med / 1e6:8.1f} GB/s",
              flush=True)
    ref = srcd["model"].cpu()
    for s in ((3, 4, 5) if a.cases == "device" else (3, 4, 5, 6, 7, 8, 9, 10)):
        assert torch.equal(slab.read(s, "model").cpu(), ref), s
    print("all slots bitwise == source")


if __name__ == "__main__":
    main()
