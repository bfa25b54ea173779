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


def _opt_worker(rank, world, port, q):
    """ShardedOptimizer over FedAdam (3 rounds, f32 + bf16 + int64 buffer that FedOPT promotes)
    and FedBuff (sharded aggregate, staleness, scale_add); oracle optimizers as the wrapped
    per-rank optimizer -- every element's arithmetic is the single-process one."""
    import torch.distributed as dist
    from oracle import oracle as O
    import scenarios as S
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ok = True
    try:
        g = torch.Generator().manual_seed(11)
        shapes = {"a": ((600, 37), torch.float32), "bf": ((5001,), torch.bfloat16), "b": ((37,), torch.float32),
                  "nbt": ((), torch.int64)}

        def model(scale):
            return {k: (torch.randn(s, generator=g) * scale).to(dt) if dt != torch.int64 else torch.tensor(5)
                    for k, (s, dt) in shapes.items()}
        w0 = model(1.0)
        hyper = dict(beta_1=0.9, beta_2=0.99, eta=1e-2, tau=1e-3)
        sharded = shard.ShardedOptimizer(O.OracleFedOPT("fedadam", **hyper), device=torch.device("cpu"))
        single = O.OracleFedOPT("fedadam", **hyper)
        ws, wr = {k: v.clone() for k, v in w0.items()}, {k: v.clone() for k, v in w0.items()}
        for r in range(3):
            n = 5
            ups = [model(1e-2) for _ in range(n)]
            for i, u in enumerate(ups):
                u["nbt"] = torch.tensor(r + i)
            counts = torch.randint(1, 100, (n,), generator=g).tolist()
            ca, cb = S.SortedCache(), S.SortedCache()
            for i in range(n):
                ca[f"t{i}"] = S.TR({k: v.clone() for k, v in ups[i].items()}, counts[i])
                cb[f"t{i}"] = S.TR({k: v.clone() for k, v in ups[i].items()}, counts[i])
            ws = sharded.do({k: v.clone() for k, v in ws.items()}, ca, total=sum(counts))
            wr = single.do({k: v.clone() for k, v in wr.items()}, cb, total=sum(counts))
            ok = ok and len(ca) == 0 and list(ws) == list(wr)
            for k in wr:
                a, b = ws[k], wr[k]
                ok = ok and a.dtype == b.dtype and a.shape == b.shape and torch.equal(
                    a.view(torch.int16) if a.dtype == torch.bfloat16 else a,
                    b.view(torch.int16) if b.dtype == torch.bfloat16 else b)
        # FedBuff: the aggregate stays sharded; scale_add gathers
        fs = shard.ShardedOptimizer(O.OracleFedBuff(), device=torch.device("cpu"), accumulate_only=True)
        fm = {k: v.clone() for k, v in w0.items() if k != "nbt"}
        fs.set_layout(fm)
        f1 = O.OracleFedBuff()
        agg_s = agg_r = None
        for i in range(4):
            u = {k: v for k, v in model(1e-2).items() if k != "nbt"}
            ca, cb = S.SortedCache(), S.SortedCache()
            ca[f"u{i}"] = S.TR({k: v.clone() for k, v in u.items()}, 3, 7 - i % 3)
            cb[f"u{i}"] = S.TR({k: v.clone() for k, v in u.items()}, 3, 7 - i % 3)
            agg_s = fs.do(agg_s, ca, total=3, version=7)
            agg_r = f1.do(agg_r, cb, total=3, version=7)
        ms, mr = {k: v.clone() for k, v in fm.items()}, {k: v.clone() for k, v in fm.items()}
        fs.scale_add_agg_weights(ms, agg_s, 4)
        f1.scale_add_agg_weights(mr, agg_r, 4)
        for k in mr:
            a, b = ms[k], mr[k]
            ok = ok and torch.equal(a.view(torch.int16) if a.dtype == torch.bfloat16 else a,
                                    b.view(torch.int16) if b.dtype == torch.bfloat16 else b)
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


def test_sharded_optimizer_fedopt_fedbuff_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_opt_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=180) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert res == {0: True, 1: True}
