import time, torch, cloudpickle, sys
from examples.mnist_aggregation import MNIST_SHAPES
from flame_amd import ingest
g = torch.Generator().manual_seed(0)
hw = {k: torch.randn(s, generator=g) * 0.05 for k, s in MNIST_SHAPES}
pls = [cloudpickle.dumps({"weights": {k: v + 1e-4*r for k, v in hw.items()}, "dataset_size": 2000}) for r in range(50)]
for p in pls[:5]: ingest.decode(p)
best = 1e9
for _ in range(5):
    t0=time.perf_counter()
    for p in pls: ingest.decode(p)
    best = min(best, (time.perf_counter()-t0)/len(pls)*1e6)
print(sys.argv[1:], "decode us/payload", round(best, 1))
