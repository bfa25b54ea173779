"""Decode time of FRESH MNIST-Net update payloads (new tensors each message, so the storage keys
inside differ): flame_amd.ingest.decode vs cloudpickle.loads.  python tools/decode_bench.py"""
import os
import sys
import time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, cloudpickle
from examples.mnist_aggregation import MNIST_SHAPES
from flame_amd import ingest
g = torch.Generator().manual_seed(0)
hw = {k: torch.randn(s, generator=g) * 0.05 for k, s in MNIST_SHAPES}
pls = [cloudpickle.dumps({"weights": {k: v + 0.01 * i for k, v in hw.items()}, "dataset_size": 2000}) for i in range(300)]
for p in pls[:20]: ingest.decode(p)
t0 = time.perf_counter()
for p in pls[20:]: ingest.decode(p)
print("decode (fresh payloads) us", (time.perf_counter() - t0) / 280 * 1e6, "records cached:", sum(len(v) for v in ingest._STORAGE_RECORDS.values()))
t0 = time.perf_counter()
for p in pls[20:120]: cloudpickle.loads(p)
print("cloudpickle.loads (fresh payloads) us", (time.perf_counter() - t0) / 100 * 1e6)
