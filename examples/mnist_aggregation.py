#!/usr/bin/env python3
"""Config 1 (examples/mnist: 2 trainers + 1 aggregator) through the MI355X path.

flame's mnist example runs a synchronous FedAvg top aggregator
(lib/python/flame/mode/horizontal/syncfl/top_aggregator.py:122-176) over two
trainers that each send ``{MessageType.WEIGHTS: state_dict, DATASET_SIZE: 2000}``
on the channel (channel.py:203-218, cloudpickle).  This script replays that round
loop without the control plane or a dataset (no network here): each "trainer"
perturbs the global MNIST ``Net`` state_dict (examples/mnist/trainer/pytorch/
main.py shapes) with synthetic deltas and pickles it exactly as the channel
would; the aggregator decodes the payload with ``flame_amd.ingest.decode``
(restricted, zero-copy), keeps it in a ``DeviceUpdateCache`` (the role's cache),
and runs the ``fedavg`` drop-in ``do(deepcopy(weights), cache, total=...)``.
Each round is checked bit for bit against the reference's own op sequence
(``tmp = (v * rate).to(v.dtype); agg += tmp`` in cache order, fedavg.py:84-104)
computed here with torch on the CPU.

    python examples/mnist_aggregation.py [--rounds 3]
"""
import argparse
import os
import sys
import time
from copy import deepcopy

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import cloudpickle  # noqa: E402
import torch  # noqa: E402

# the MNIST example's Net (conv1 1->32 3x3, conv2 32->64 3x3, fc1 9216->128, fc2 128->10)
MNIST_SHAPES = [("conv1.weight", (32, 1, 3, 3)), ("conv1.bias", (32,)), ("conv2.weight", (64, 32, 3, 3)),
                ("conv2.bias", (64,)), ("fc1.weight", (128, 9216)), ("fc1.bias", (128,)),
                ("fc2.weight", (10, 128)), ("fc2.bias", (10,))]


class TrainResult:
    """lib/python/flame/optimizer/train_result.py:19-26."""

    def __init__(self, weights=None, count=0, version=0):
        self.weights, self.count, self.version = weights, count, version


def reference_fedavg(base, updates):
    """fedavg.py:79-104 as the reference computes it (torch CPU, cache order)."""
    agg = {k: v.clone() for k, v in base.items()}
    total = sum(c for _, c in updates)
    for w, c in updates:
        rate = c / total
        for k, v in w.items():
            agg[k] += (v * rate).to(v.dtype)
    return agg


def run(rounds: int = 3, seed: int = 0, verbose: bool = True) -> bool:
    from flame_amd import ingest
    from flame_amd.optimizers import optimizer_provider

    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(seed)
    weights = {k: torch.randn(s, generator=g) * 0.05 for k, s in MNIST_SHAPES}     # the top's global model
    host_weights = {k: v.clone() for k, v in weights.items()}
    weights = {k: v.to(dev) for k, v in weights.items()}
    optimizer = optimizer_provider.get("fedavg")
    # the role's self.cache lives across rounds (syncfl/top_aggregator.py internal init)
    cache = ingest.DeviceUpdateCache(device=dev, placement="hbm", capacity=4)
    ok = True
    for rnd in range(rounds):
        # trainers: train (here: a synthetic delta) and send {WEIGHTS, DATASET_SIZE} on the channel
        payloads, sent = [], []
        for t in range(2):
            local = {k: v + torch.randn(v.shape, generator=g) * 1e-2 for k, v in host_weights.items()}
            payloads.append((f"trainer{t}", cloudpickle.dumps({"weights": local, "dataset_size": 2000})))
            sent.append((local, 2000))
        # aggregator: recv_fifo -> cache[end] = TrainResult(weights, count); total = Σ count
        t0 = time.perf_counter()
        total = 0
        for end, payload in payloads:
            msg = ingest.decode(payload)
            total += msg["dataset_size"]
            cache[end] = TrainResult(msg["weights"], msg["dataset_size"])
        weights = optimizer.do(deepcopy(weights), cache, total=total, num_trainers=2)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        ref = reference_fedavg(host_weights, sent)
        same = all(torch.equal(weights[k].cpu(), ref[k]) for k in ref)
        ok = ok and same
        host_weights = ref
        if verbose:
            print(f"round {rnd}: aggregated 2 x {sum(v.numel() for v in ref.values())} params in {dt * 1e3:.2f} ms "
                  f"(decode + cache + FedAvg), bitwise == reference op sequence: {same}")
    return ok


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    sys.exit(0 if run(args.rounds) else 1)


if __name__ == "__main__":
    main()
