#!/usr/bin/env python3
"""FedDyn round kernel: history layout A/B (contiguous rows vs tiled like the UpdateSlab),
updated in place or written to a second buffer (ping-pong).

One process, interleaved rounds, 512 ends x 25M fp32, every end tracked and arriving
(the merged one-pass program: read w, read h, write h', avg, mean).  Arrivals are
tiled ([tiles][N][T]) in both variants.  Prints kernel ms and algorithmic GB/s.

    python tools/feddyn_layout.py [--clients 512 --params 25000000 --rounds 5]
"""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=512)
    ap.add_argument("--params", type=int, default=25_000_000)
    ap.add_argument("--rounds", type=int, default=5)
    args = ap.parse_args()
    import torch
    from flame_amd import _native as N
    from flame_amd import engine
    dev = torch.device("cuda", 0)
    n, P = args.clients, args.params
    code = N.FLAME_F32
    T = engine.chunk_elems(code)
    tiles = -(-P // T)
    w = torch.empty((tiles, n, T), dtype=torch.float32, device=dev)
    engine.synth_fill_(w.view(-1), 3, 1, 0, 1e-2)
    h_rows = torch.empty((n, tiles * T), dtype=torch.float32, device=dev)
    engine.synth_fill_(h_rows.view(-1), 3, 2, 0, 1e-2)
    h_tiled = torch.empty((tiles, n, T), dtype=torch.float32, device=dev)
    engine.synth_fill_(h_tiled.view(-1), 3, 2, 0, 1e-2)
    # second history buffers: the updated history written to a different address (ping-pong)
    h_rows2 = torch.empty_like(h_rows)
    h_tiled2 = torch.empty_like(h_tiled)
    base = torch.empty(P, dtype=torch.float32, device=dev)
    engine.synth_fill_(base, 3, 0, 0, 1.0)
    out = torch.empty_like(base)
    cld = torch.empty_like(base)
    f = N.FLAME_DYN_W | N.FLAME_DYN_AVG | N.FLAME_DYN_HIN | N.FLAME_DYN_HOUT | N.FLAME_DYN_MEAN
    flags = [f] * n
    wp = [w[0, i].data_ptr() for i in range(n)]
    variants = {
        "rows": engine.DynSeg(P, out=out.data_ptr(), inp=base.data_ptr(), cld=cld.data_ptr(),
                              steps=[(wp[i], h_rows[i].data_ptr(), h_rows[i].data_ptr()) for i in range(n)],
                              tile_stride=n * T * 4),
        "tiled": engine.DynSeg(P, out=out.data_ptr(), inp=base.data_ptr(), cld=cld.data_ptr(),
                               steps=[(wp[i], h_tiled[0, i].data_ptr(), h_tiled[0, i].data_ptr()) for i in range(n)],
                               tile_stride=n * T * 4, hist_tile_stride=n * T * 4),
        "rows_pingpong": engine.DynSeg(P, out=out.data_ptr(), inp=base.data_ptr(), cld=cld.data_ptr(),
                                       steps=[(wp[i], h_rows[i].data_ptr(), h_rows2[i].data_ptr()) for i in range(n)],
                                       tile_stride=n * T * 4),
        "tiled_pingpong": engine.DynSeg(P, out=out.data_ptr(), inp=base.data_ptr(), cld=cld.data_ptr(),
                                        steps=[(wp[i], h_tiled[0, i].data_ptr(), h_tiled2[0, i].data_ptr())
                                               for i in range(n)],
                                        tile_stride=n * T * 4, hist_tile_stride=n * T * 4),
    }
    nbytes = (3 * n + 3) * P * 4
    times = {k: [] for k in variants}
    keep = []
    for r in range(args.rounds + 1):
        for name, seg in variants.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            engine.feddyn_round_(code, [seg], flags, n, 1.0 / n, 1.0 / n, dev, keep)
            e1.record()
            torch.cuda.synchronize()
            if r:
                times[name].append(e0.elapsed_time(e1))
        keep.clear()
    # read-2 / write-1 streaming reference: torch's h += w over the same bytes (3 x n x P x 4)
    hv, wv = h_rows.view(-1), w.view(-1)[:h_rows.numel()]
    tt = []
    for r in range(args.rounds + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        hv.add_(wv)
        e1.record()
        torch.cuda.synchronize()
        if r:
            tt.append(e0.elapsed_time(e1))
    med = statistics.median(tt)
    print(f"torch h.add_(w) (2 reads : 1 write) median {med:8.3f} ms  {3 * hv.numel() * 4 / med / 1e6:8.1f} GB/s")
    for name, ts in times.items():
        med = statistics.median(ts)
        print(f"{name:6s} median {med:8.3f} ms  min {min(ts):8.3f} ms  {nbytes / med / 1e6:8.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
