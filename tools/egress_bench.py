#!/usr/bin/env python3
"""Egress: the aggregated model (device-resident) as the payload sent back to N trainers.

reference: per end, weights_to_device(self.weights, CPU) + cloudpickle.dumps (channel.send),
           syncfl/top_aggregator.py:184-215, channel.py:203-218;
flame_amd: ONE MessageEncoder.encode (tensors D2H straight into the pinned payload), the same
           payload handed to every end (+ one bytes() copy when the backend needs bytes).

    python tools/egress_bench.py [--params 25000000] [--ends 4]
"""
import argparse
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import cloudpickle
    from flame_amd import egress
    ap = argparse.ArgumentParser()
    ap.add_argument("--params", type=int, default=25_000_000)
    ap.add_argument("--ends", type=int, default=4)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    model = {"model": torch.randn(a.params, device=dev)}
    meta = {"round": 3, "datasampler": {"e": [1, 2]}}
    enc = egress.MessageEncoder(ring=2)

    def reference():
        out = []
        for _ in range(a.ends):
            w = {k: v.to("cpu") for k, v in model.items()}          # weights_to_device(self.weights, CPU)
            out.append(cloudpickle.dumps({"weights": w, **meta}))
        return out

    def ours():
        pl = enc.encode({"weights": model, **meta})
        return [pl] * a.ends

    def ours_bytes():
        pl = enc.encode_bytes({"weights": model, **meta})
        return [pl] * a.ends

    res = {}
    for name, fn in (("reference (D2H + cloudpickle.dumps per end)", reference), ("flame_amd encode once (memoryview)", ours),
                     ("flame_amd encode once + bytes()", ours_bytes)):
        fn()
        ts = []
        for _ in range(a.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        res[name] = statistics.median(ts)
        print(f"{name:48s} {res[name] * 1e3:9.2f} ms for {a.ends} ends ({a.params * 4 / 1e6:.0f} MB model)", flush=True)
    back = cloudpickle.loads(bytes(ours()[0]))
    assert torch.equal(back["weights"]["model"], model["model"].cpu())
    print("payload loads back bitwise")


if __name__ == "__main__":
    main()
