#!/usr/bin/env python3
"""Can two RCCL ranks share ONE GPU (so the world>1 collective path runs on a 1-GPU box)?
Each rank: set_device(0), init nccl, an in-place all_gather_into_tensor under
_coalescing_manager and a public one, checked.  Launch:
  python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \
      tools/rccl_one_gpu_probe.py"""
import os

import torch
import torch.distributed as dist


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    n = 1 << 20
    out = torch.full((world * n,), -1.0, device="cuda")
    out[rank * n:(rank + 1) * n] = rank + 1.0
    dist.all_gather_into_tensor(out, out[rank * n:(rank + 1) * n])
    torch.cuda.synchronize()
    ok1 = all(bool((out[r * n:(r + 1) * n] == r + 1.0).all()) for r in range(world))
    from torch.distributed.distributed_c10d import _coalescing_manager
    a = torch.full((world * 4096,), -1.0, device="cuda")
    b = torch.full((world * 100,), -1, dtype=torch.float32, device="cuda")
    a[rank * 4096:(rank + 1) * 4096] = 10.0 + rank
    b[rank * 100:(rank + 1) * 100] = 20.0 + rank
    with _coalescing_manager(device=torch.device("cuda", 0), async_ops=True) as cm:
        dist.all_gather_into_tensor(a, a[rank * 4096:(rank + 1) * 4096])
        dist.all_gather_into_tensor(b, b[rank * 100:(rank + 1) * 100])
    cm.wait()
    torch.cuda.synchronize()
    ok2 = all(bool((a[r * 4096:(r + 1) * 4096] == 10.0 + r).all()) and bool((b[r * 100:(r + 1) * 100] == 20.0 + r).all())
              for r in range(world))
    print(f"rank {rank}: public in-place all-gather {'ok' if ok1 else 'WRONG'}, coalesced {'ok' if ok2 else 'WRONG'}",
          flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
