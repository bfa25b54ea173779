#!/usr/bin/env python3
"""Config 5 shard, one process: middle weights as 64 separate tensors (rows) vs as the slots
of one tiled UpdateSlab ([tiles][64][T]: a chunk's 64 middles are one contiguous block).

Rounds alternate between the two layouts from identical state; every pair is checked
bitwise (top weights, top aggregate, middle weights); kernel time from HIP events on the
launch stream.  A read probe over the same arrival slab gives the same-run ceiling.

    python tools/hier_midlayout.py --rounds 6
"""
import argparse
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class Cache(dict):
    def iterkeys(self):
        return iter(sorted(self))


class TR:
    def __init__(self, w, c, v=0):
        self.weights, self.count, self.version = w, c, v


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--mids", type=int, default=64)
    ap.add_argument("--clients", type=int, default=64)
    ap.add_argument("--params", type=int, default=15_625_000)
    ap.add_argument("--fetched", action="store_true", help="read-only middles (no write-back)")
    a = ap.parse_args()
    from flame_amd import engine, synth
    from flame_amd.optimizer.fedbuff import FedBuff, hierarchy_round
    from flame_amd.slab import UpdateSlab
    dev = torch.device("cuda", 0)
    M, C, P, dt, rnd = a.mids, a.clients, a.params, torch.bfloat16, 10
    store = UpdateSlab({"model": torch.empty(P, dtype=dt)}, capacity=M * C, device=dev)
    tmp = torch.empty(P, dtype=dt, device=dev)
    ws = []
    for i in range(M * C):
        engine.synth_fill_(tmp, 6, 1 + i, 0, 1e-2)
        ws.append(store.put({"model": tmp}))
    rows = []
    for m in range(M):
        engine.synth_fill_(tmp, 6, 10_000 + m, 0, 1.0)
        rows.append({"model": tmp.clone()})
    mslab = UpdateSlab({"model": torch.empty(P, dtype=dt)}, capacity=M, device=dev)
    tiled = [mslab.put(r) for r in rows]
    engine.synth_fill_(tmp, 6, 0, 0, 1.0)
    top = {"row": {"model": tmp.clone()}, "tiled": {"model": tmp.clone()}}
    del tmp
    stale = [int(x) % 4 for x in synth.counts(6, M * C)]
    mids = {"row": rows, "tiled": tiled}
    times = {"row": [], "tiled": []}
    torch.cuda.synchronize()
    for r in range(a.rounds + 1):
        outs = {}
        for lay in ("row", "tiled") if r % 2 == 0 else ("tiled", "row"):
            aggs = [None] * M
            opts = [FedBuff() for _ in range(M)]
            for m in range(M):
                for t in range(C):
                    c = Cache()
                    c[f"{m * C + t:05d}"] = TR(ws[m * C + t], 1, rnd - stale[m * C + t])
                    aggs[m] = opts[m].do(aggs[m], c, total=1, version=rnd)
            engine.kernel_events = []
            agg, _ = hierarchy_round([(mids[lay][m], aggs[m], C, rnd - m % 2) for m in range(M)], None, version=rnd,
                                     top_weights=top[lay], top_goal=M, update_middle_weights=not a.fetched)
            ev = engine.kernel_events
            engine.kernel_events = None
            torch.cuda.synchronize()
            assert [e[0] for e in ev] == ["flame_hier_fedbuff"], [e[0] for e in ev]
            t = ev[0][1].elapsed_time(ev[0][2]) / 1e3
            if r:
                times[lay].append((t, ev[0][3]))
            outs[lay] = agg["model"].clone()
        assert torch.equal(outs["row"].view(torch.int16), outs["tiled"].view(torch.int16)), "top agg differs"
        assert torch.equal(top["row"]["model"].view(torch.int16), top["tiled"]["model"].view(torch.int16))
    for m in range(M):
        assert torch.equal(rows[m]["model"].view(torch.int16),
                           mslab.read(tiled[m].slot, "model").reshape(-1).view(torch.int16)), f"middle {m}"
    for lay, ts in times.items():
        med = statistics.median(t for t, _ in ts)
        print(f"{lay:6s} middles: kernel median {med * 1e3:.3f} ms over {len(ts)} rounds "
              f"({', '.join(f'{t * 1e3:.2f}' for t, _ in ts)}), {ts[0][1] / med / 1e9:.0f} GB/s algorithmic",
              flush=True)
    print("bitwise: top weights, top aggregate and middle weights equal across layouts", flush=True)


if __name__ == "__main__":
    main()
