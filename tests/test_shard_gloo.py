"""Parameter-sharded FedAvg over a world_size-2 gloo group on CPU.

The partition + all-gather logic of flame_amd.shard must reproduce the
single-process reference result bitwise; the per-rank reducer is the oracle
here (no GPU), the HIP kernel in the product path.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from flame_amd import shard


def test_shard_bounds_aligned_and_covering():
    for numel in [0, 1, 1023, 1024, 25_000_000, 1_199_882]:
        for world in [1, 2, 3, 8]:
            for isz in [2, 4, 8]:
                b = shard.shard_bounds(numel, world, isz)
                assert len(b) == world and b[0][0] == 0 and b[-1][1] == numel
                for (l0, h0), (l1, h1) in zip(b, b[1:]):
                    assert h0 == l1
                for lo, _ in b:
                    assert (lo * isz) % 4096 == 0 or lo == numel


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    from oracle import oracle as O
    import scenarios as S
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(7)
        shapes = {"a": (1000, 37), "b": (37,), "c": (5000,), "h": (3001,)}
        dts = {"a": torch.float32, "b": torch.float32, "c": torch.bfloat16, "h": torch.float32}
        base = {k: torch.randn(s, generator=g).to(dts[k]) for k, s in shapes.items()}
        n = 11
        clients = [{k: (torch.randn(s, generator=g) * 1e-2).to(dts[k]) for k, s in shapes.items()} for _ in range(n)]
        counts = torch.randint(1, 1000, (n,), generator=g).tolist()
        cache = S.SortedCache()
        for i in range(n):
            cache[f"{i:02d}"] = S.TR(clients[i], counts[i])

        def oracle_reducer(acc, cl, rates):
            O.reduce_tensor(acc, cl, rates)
        sf = shard.ShardedFedAvg(device=torch.device("cpu"), reducer=oracle_reducer)
        mine = {k: v.clone() for k, v in base.items()}
        out = sf.do(mine, cache, total=sum(counts))
        assert out is mine and len(cache) == 0
        # single-process oracle FedAvg
        ref = {k: v.clone() for k, v in base.items()}
        c2 = S.SortedCache()
        for i in range(n):
            c2[f"{i:02d}"] = S.TR(clients[i], counts[i])
        O.OracleFedAvg().do(ref, c2, total=sum(counts))
        ok = all(torch.equal(out[k].view(torch.int16) if out[k].dtype == torch.bfloat16 else out[k],
                             ref[k].view(torch.int16) if ref[k].dtype == torch.bfloat16 else ref[k]) for k in ref)
        # slice mode + pipelined gather: each rank gets only its slice of one flat vector
        P = 10_000
        glob_base = torch.randn(P * world, generator=g)
        glob_cl = [torch.randn(P * world, generator=g) * 1e-2 for _ in range(n)]
        fr = (0.75, 0.2, 0.05)
        pieces = shard.piece_bounds(P, fr, 1024)

        def local(v):  # rank's local slice in piece-major global order
            return torch.cat([v[world * lo + rank * (hi - lo): world * lo + (rank + 1) * (hi - lo)] for lo, hi in pieces])
        ss = shard.ShardedSliceFedAvg(fracs=fr, reducer=oracle_reducer)
        c3 = S.SortedCache()
        for i in range(n):
            c3[f"{i:02d}"] = S.TR({"m": local(glob_cl[i])}, counts[i])
        lb = {"m": local(glob_base)}
        ss.do(lb, c3, total=sum(counts))
        ref3 = glob_base.clone()
        O.reduce_tensor(ref3, glob_cl, [c / sum(counts) for c in counts])
        ok = ok and torch.equal(ss.global_flat, ref3) and torch.equal(lb["m"], local(ref3))
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


def test_sharded_fedavg_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=180) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert res == {0: True, 1: True}


def test_piece_bounds():
    assert shard.piece_bounds(10_000, (0.75, 0.2, 0.05), 1024) == [(0, 7168), (7168, 9216), (9216, 10_000)]
    assert shard.piece_bounds(100, (0.75, 0.2, 0.05), 1024) == [(0, 100)]
    b = shard.piece_bounds(25_000_000, (0.75, 0.2, 0.05), 1024)
    assert b[0][0] == 0 and b[-1][1] == 25_000_000 and all(lo % 1024 == 0 for lo, _ in b)
