#!/usr/bin/env python3
"""Host -> HBM copy paths for one update, on the MI355X: which way into the tiled slab keeps PCIe
busy for a hipHostRegister-ed POSIX shared-memory segment (the LIFL receive buffer) vs a torch
pinned tensor.  Each path copies the same bytes into a (tiles, 4 KiB) tiled destination (or a
contiguous one for the plain copy), median of --reps, GB/s; the destination is checked bytewise.

    python tools/h2d_paths.py [--mb 100] [--reps 5]
"""
import argparse
import os
import statistics
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=100)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--offsets", default="0,4,356", help="source byte offsets into the buffers (a pickled update's "
                                                         "storage starts a few hundred bytes in, at no particular alignment)")
    a = ap.parse_args()
    from multiprocessing import shared_memory
    from flame_amd import _native as N, engine, ingest
    L = N.lib()
    nbytes = a.mb << 20
    dev = torch.device("cuda", 0)
    pad = 4096
    pinned_all = torch.empty(nbytes + pad, dtype=torch.uint8, pin_memory=True)
    pinned_all.copy_(torch.from_numpy(np.random.default_rng(1).integers(0, 255, nbytes + pad, dtype=np.uint8)))
    seg = shared_memory.SharedMemory(create=True, size=nbytes + pad)
    try:
        shm_all = torch.frombuffer(seg.buf, dtype=torch.uint8)
        shm_all.copy_(pinned_all)
        reg = ingest.RegisteredBuffer(seg.buf)
        T = N.FLAME_TILE_BYTES
        tiles = nbytes // T
        stride = T * 3                                   # a slot of a 3-client slab: tile stride 3 x 4 KiB
        dst = torch.empty(tiles * stride, dtype=torch.uint8, device=dev)
        flat = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        st = torch.cuda.current_stream(dev)

        def table(src_ptr):
            t = np.asarray([(src_ptr, dst.data_ptr(), nbytes, stride)], dtype=np.int64)
            return t

        def run(fn):
            ts = []
            for _ in range(a.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn()
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1) / 1e3)
            return nbytes / statistics.median(ts) / 1e9

        def check_tiled(ref):
            got = dst.view(tiles, stride)[:, :T].reshape(-1).cpu()
            return bool(torch.equal(got, ref))

        def paths_at(off):
            pinned, shm = pinned_all[off:off + nbytes], shm_all[off:off + nbytes]
            paths = {
                f"+{off} B pinned: contiguous copy_ (hipMemcpyAsync)":
                    (lambda: flat.copy_(pinned, non_blocking=True), None),
                f"+{off} B shm registered: contiguous copy_": (lambda: flat.copy_(shm, non_blocking=True), None),
            }
            for nm, src in ((f"+{off} B pinned", pinned), (f"+{off} B shm registered", shm)):
                tb = table(src.data_ptr())
                paths[f"{nm}: flame_slab_write_2d (hipMemcpy2DAsync, 4 KiB rows)"] = (
                    lambda tb=tb: N.check(L.flame_slab_write_2d(tb.ctypes.data, 1, st.cuda_stream)), check_tiled)
                tbd = table(engine.host_device_pointer(src.data_ptr()))
                paths[f"{nm}: flame_slab_write kernel over the device-mapped pointer"] = (
                    lambda tbd=tbd: N.check(L.flame_slab_write(tbd.ctypes.data, 1, st.cuda_stream)), check_tiled)
            return pinned, paths

        for off in [int(x) for x in a.offsets.split(",")]:
            pinned, paths = paths_at(off)
            for nm, (fn, chk) in paths.items():
                dst.zero_()
                r = run(fn)
                ok = chk(pinned) if chk else bool(torch.equal(flat.cpu(), pinned))
                print(f"{nm:72s} {r:7.2f} GB/s  {'ok' if ok else 'MISMATCH'}", flush=True)
        reg.close()
        del shm_all, paths
    finally:
        seg.close()
        seg.unlink()


if __name__ == "__main__":
    main()
