"""Parameter sharding (flame_amd.shard) over world-size-2 gloo groups on CPU.

The all-gathers run the same code RCCL runs (``_Comm.all_gather_inplace``: async, in place,
one coalesced group per wave; gloo accepts it for CPU tensors) -- the workers check that no
host-staged gather happened.

The plan / slicing / replay / in-place all-gather logic of ShardedOptimizer and
ShardedHierarchy must reproduce the single-process result bitwise.  The per-rank
arithmetic is the oracle here (no GPU); the product runs the HIP drop-ins per rank
(tests/test_gpu_parity.py runs the same compositions with two ranks on the GPU).
A small ``align`` makes the tiny fixture models shard (the product default is 2048).
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from flame_amd import shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(target, world=2, timeout=180):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=target, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=timeout) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert res == {r: True for r in range(world)}, res


def _init(rank, world, port):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    return dist


def _eq(a, b):
    if a.dtype != b.dtype or a.shape != b.shape:
        return False
    if a.dtype in (torch.bfloat16, torch.float16):
        return torch.equal(a.view(torch.int16), b.view(torch.int16))
    return torch.equal(a, b)


def _model(g, shapes, scale):
    def one(s, dt):
        if dt.is_floating_point:
            return (torch.randn(s, generator=g) * scale).to(dt)
        if s == ():
            return torch.tensor(5, dtype=dt)
        return torch.randint(0, 2 if dt == torch.bool else 120, s, generator=g).to(dt)
    return {k: one(s, dt) for k, (s, dt) in shapes.items()}


# ---------------------------------------------------------------- the plan (no process group)
@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("align", [8, 2048])
def test_shard_plan_partitions_every_key(world, align):
    shapes = {"conv": ((32, 1, 3, 3), torch.float32), "bias": ((32,), torch.float32),
              "fc1": ((128, 9216), torch.float32), "big": ((3, 1_000_003), torch.bfloat16),
              "nbt": ((), torch.int64), "fc2": ((10, 128), torch.float16), "empty": ((0, 4), torch.float32)}
    model = {k: torch.empty(s, dtype=dt, device="meta") for k, (s, dt) in shapes.items()}
    plans = [shard.ShardPlan(model, world, r, align=align) for r in range(world)]
    unit = world * align
    for k, t in model.items():
        n = t.numel()
        cover = torch.zeros(n, dtype=torch.int32)
        for p in plans:
            for s in p.subs:
                if s.key != k:
                    continue
                if s.tail:
                    assert (s.lo, s.hi) == (s.g0, s.g1) and s.g0 == n // unit * unit and s.wave == 0
                    if p.rank == 0:
                        cover[s.lo:s.hi] += 1
                else:
                    assert (s.g1 - s.g0) % unit == 0 and s.lo % align == 0 and (s.hi - s.lo) * world == s.g1 - s.g0
                    assert s.lo == s.g0 + p.rank * (s.hi - s.lo)
                    cover[s.lo:s.hi] += 1
        assert bool((cover == 1).all()), k
    for p in plans:   # the same local names on every rank; waves are 1..3 and non-empty
        assert p.names == plans[0].names and 1 <= p.n_waves <= 3 and all(p.wave_names)
        assert sum(len(w) for w in p.wave_names) == len(p.names)
        assert p.owned_elements() == sum(p.local_numel.values())
    # wave sizes follow the 75 / 20 / 5 split of the main parts
    if align == 2048 and world == 8:
        sizes = [sum(plans[0].by_name[n].g1 - plans[0].by_name[n].g0 for n in w if not plans[0].by_name[n].tail)
                 for w in plans[0].wave_names]
        assert sizes[0] > sizes[1] > sizes[2] > 0


def test_shard_plan_slices_and_restrict():
    g = torch.Generator().manual_seed(3)
    w = {"a": torch.randn(100, 37, generator=g), "b": torch.randn(37, generator=g)}
    p = shard.ShardPlan(w, 2, 1, align=8)
    loc = p.slice_update(w)
    assert list(loc) == p.names
    for n, v in loc.items():
        s = p.by_name[n]
        assert torch.equal(v, w[s.key].reshape(-1)[s.lo:s.hi])
    for wave in range(p.n_waves):
        r = p.restrict(loc, wave)
        assert list(r) == p.wave_names[wave]
    with pytest.raises(KeyError):
        p.slice_update({"a": w["a"], "zz": w["b"]})
    # no process group: a ShardedOptimizer is a world-1 pass-through that still shards into waves
    from oracle import oracle as O
    import scenarios as S
    opt = shard.ShardedOptimizer(O.OracleFedAvg(), device=torch.device("cpu"), waves=True, align=8)
    c1, c2 = S.SortedCache(), S.SortedCache()
    ups = [{k: v * 1e-2 + i for k, v in w.items()} for i in range(3)]
    for i, u in enumerate(ups):
        c1[f"{i}"] = S.TR({k: v.clone() for k, v in u.items()}, 5 + i)
        c2[f"{i}"] = S.TR({k: v.clone() for k, v in u.items()}, 5 + i)
    a = {k: v.clone() for k, v in w.items()}
    b = {k: v.clone() for k, v in w.items()}
    assert opt.do(a, c1, total=18) is a and len(c1) == 0
    O.OracleFedAvg().do(b, c2, total=18)
    assert all(_eq(a[k], b[k]) for k in w)
    assert opt.do(a, S.SortedCache(), total=18) is None


# ---------------------------------------------------------------- FedAvg (waves) / FedOPT / FedBuff
SHAPES = {"a": ((600, 37), torch.float32), "bf": ((5001,), torch.bfloat16), "b": ((37,), torch.float32),
          "nbt": ((), torch.int64), "h": ((3001,), torch.float16)}
# FedAvg also carries a bool mask and a uint8 buffer (split across ranks like any key)
FEDAVG_SHAPES = {**SHAPES, "mask": ((4099,), torch.bool), "u8": ((2500,), torch.uint8)}


def _fedavg_worker(rank, world, port, q):
    dist = _init(rank, world, port)
    try:
        from oracle import oracle as O
        import scenarios as S
        g = torch.Generator().manual_seed(7)
        base = _model(g, FEDAVG_SHAPES, 1.0)
        ok = True
        opt = shard.ShardedOptimizer(O.OracleFedAvg(), device=torch.device("cpu"), align=8, waves=True)
        for r in range(2):
            n = 11
            clients = [_model(g, FEDAVG_SHAPES, 1e-2) for _ in range(n)]
            for i, c in enumerate(clients):
                c["nbt"] = torch.tensor(r + i)
            counts = torch.randint(1, 1000, (n,), generator=g).tolist()
            ca, cb = S.SortedCache(), S.SortedCache()
            for i in range(n):
                ca[f"{i:02d}"] = S.TR({k: v.clone() for k, v in clients[i].items()}, counts[i])
                cb[f"{i:02d}"] = S.TR({k: v.clone() for k, v in clients[i].items()}, counts[i])
            mine = {k: v.clone() for k, v in base.items()}
            out = opt.do(mine, ca, total=sum(counts), num_trainers=n)
            ok = ok and out is mine and len(ca) == 0 and opt.plan.n_waves == 3
            ref = {k: v.clone() for k, v in base.items()}
            O.OracleFedAvg().do(ref, cb, total=sum(counts))
            ok = ok and all(_eq(out[k], ref[k]) for k in ref)
            base = ref
        # the gathers ran the body RCCL runs (async, in place; coalesced per wave unless disabled)
        st = shard.GATHER_STATS
        ok = ok and st["host_staged"] == 0 and st["coalesced"] + st["async"] > 0
        ok = ok and (st["coalesced"] > 0 if shard.COALESCE and world == 2 else True)
        ok = ok and (st["coalesced"] == 0 if not shard.COALESCE else True)
        # None results (fedavg.py:76-77)
        ok = ok and opt.do({k: v.clone() for k, v in base.items()}, S.SortedCache(), total=3) is None
        c = S.SortedCache()
        c["x"] = S.TR({k: v.clone() for k, v in base.items()}, 0)
        ok = ok and opt.do({k: v.clone() for k, v in base.items()}, c, total=0) is None
        q.put((rank, bool(ok)))
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def test_sharded_fedavg_waves_gloo_world2():
    _run(_fedavg_worker)


def _fedavg_worker_public(rank, world, port, q):
    shard.COALESCE = False        # FLAME_AMD_COALESCE=0: one public async all-gather per piece
    _fedavg_worker(rank, world, port, q)


def test_sharded_fedavg_waves_gloo_world2_public_collectives():
    """The same rounds without torch's private coalescing helper (the fallback path)."""
    _run(_fedavg_worker_public)


def _opt_worker(rank, world, port, q):
    """ShardedOptimizer over FedAdam (3 rounds + an empty round, f32 / bf16 / f16 + an int64
    buffer that FedOPT promotes) and FedBuff (sharded aggregate, staleness, scale_add)."""
    dist = _init(rank, world, port)
    ok = True
    try:
        from oracle import oracle as O
        import scenarios as S
        g = torch.Generator().manual_seed(11)
        w0 = _model(g, SHAPES, 1.0)
        hyper = dict(beta_1=0.9, beta_2=0.99, eta=1e-2, tau=1e-3)
        sharded = shard.ShardedOptimizer(O.OracleFedOPT("fedadam", **hyper), device=torch.device("cpu"), align=8)
        single = O.OracleFedOPT("fedadam", **hyper)
        ws, wr = {k: v.clone() for k, v in w0.items()}, {k: v.clone() for k, v in w0.items()}
        for r in range(3):
            n = 5
            ups = [_model(g, SHAPES, 1e-2) for _ in range(n)]
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
            ok = ok and all(_eq(ws[k], wr[k]) for k in wr)
        # an empty round returns the previous round's (full-model) result, as the reference
        # returns current_weights (fedopt.py:84-85)
        again = sharded.do({k: v.clone() for k, v in ws.items()}, S.SortedCache(), total=7)
        ok = ok and again is ws and all(again[k].shape == w0[k].shape for k in w0)
        # FedBuff: the aggregate stays sharded; scale_add gathers in place
        fm = {k: v.clone() for k, v in w0.items() if k != "nbt"}
        fs = shard.ShardedOptimizer(O.OracleFedBuff(), device=torch.device("cpu"), accumulate_only=True, align=8)
        fs.set_layout(fm)
        f1 = O.OracleFedBuff()
        agg_s = agg_r = None
        for i in range(4):
            u = {k: v for k, v in _model(g, SHAPES, 1e-2).items() if k != "nbt"}
            ca, cb = S.SortedCache(), S.SortedCache()
            ca[f"u{i}"] = S.TR({k: v.clone() for k, v in u.items()}, 3, 7 - i % 3)
            cb[f"u{i}"] = S.TR({k: v.clone() for k, v in u.items()}, 3, 7 - i % 3)
            agg_s = fs.do(agg_s, ca, total=3, version=7)
            agg_r = f1.do(agg_r, cb, total=3, version=7)
        ok = ok and list(agg_s) == fs.plan.names
        ms, mr = {k: v.clone() for k, v in fm.items()}, {k: v.clone() for k, v in fm.items()}
        out = fs.scale_add_agg_weights(ms, agg_s, 4)
        f1.scale_add_agg_weights(mr, agg_r, 4)
        ok = ok and out is ms and all(_eq(ms[k], mr[k]) for k in mr)
        st = shard.GATHER_STATS
        ok = ok and st["host_staged"] == 0 and st["coalesced"] + st["async"] > 0
        q.put((rank, bool(ok)))
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def test_sharded_optimizer_fedopt_fedbuff_gloo_world2():
    _run(_opt_worker)


# ---------------------------------------------------------------- config 5: the sharded hierarchy
def _hier_worker(rank, world, port, q):
    """ShardedHierarchy (oracle per-rank hierarchy) on the reference-generated
    hier_fedbuff_small fixture: top model == the fixture's (bitwise) on every rank, each
    rank's middle deltas == its slices of the fixture's deltas; and the synchronous round
    on hier_fedavg_small (f32 / bf16 / f16 / int64, 2 rounds)."""
    dist = _init(rank, world, port)
    ok = True
    try:
        from fixture_io import Fixture
        from oracle import oracle as O
        import scenarios as S
        gold = os.path.join(os.path.dirname(__file__), "golden")
        fx = Fixture(os.path.join(gold, "hier_fedbuff_small.npz"))
        rnd = fx.meta["round"]
        top_w0 = fx.weights("top_w0")
        hier = shard.ShardedHierarchy(top_w0, device=torch.device("cpu"), align=8,
                                      round_fn=S.oracle_hierarchy_round)
        ok = ok and hier.plan.n_waves == 2 and any(not s.tail for s in hier.plan.subs)
        middles = []
        for mid in range(2):
            opt, agg = hier.middle_optimizer(O.OracleFedBuff()), None
            for t in range(3):
                c = S.SortedCache()
                c[f"m{mid}t{t}"] = S.TR(fx.weights(f"m{mid}/update{t}"), 10 + t, rnd - t % 2)
                agg = opt.do(agg, c, total=10 + t, version=rnd)
            middles.append(({k: v.clone() for k, v in top_w0.items()}, agg, 3, rnd - mid))
        top = {k: v.clone() for k, v in top_w0.items()}
        top_agg, deltas = hier.round(middles, None, version=rnd, top_weights=top, top_goal=2, with_delta=True)
        ok = ok and all(_eq(top[k], fx.weights("top_out")[k]) for k in top)
        ok = ok and list(top_agg) == hier.plan.names
        for mid in range(2):
            exp = hier.plan.slice_update(fx.weights(f"m{mid}/delta"))
            ok = ok and all(_eq(deltas[mid][n], exp[n]) for n in exp)

        # synchronous hierarchy (syncfl middles -> syncfl top) vs the reference fixture
        fs = Fixture(os.path.join(gold, "hier_fedavg_small.npz"))
        m = fs.meta
        tw = fs.weights("top_w0")
        hs = shard.ShardedHierarchy(tw, device=torch.device("cpu"), align=8,
                                    sync_round_fn=S.oracle_sync_hierarchy_round)
        top = {k: v.clone() for k, v in tw.items()}
        mids = [{k: v.clone() for k, v in tw.items()} for _ in range(3)]
        for r, rm in enumerate(m["rounds"]):
            specs = []
            for j, mm in enumerate(rm["mids"]):
                cache = S.SortedCache()
                for i, (e, c) in enumerate(zip(mm["ids"], mm["counts"])):
                    cache[e] = S.TR(fs.weights(f"r{r}/m{j}/client{i}"), c)
                specs.append((mids[j], cache, sum(mm["counts"])))
            out, _ = hs.sync_round(specs, top)
            ok = ok and out is top and all(_eq(top[k], fs.weights(f"r{r}/top")[k]) for k in top)
            ok = ok and shard.GATHER_STATS["host_staged"] == 0
            # keys whose middle weights this rank updated in full (the tails) match the reference
            for j in range(3):
                exp = hs.plan.slice_update(fs.weights(f"r{r}/m{j}/new"))
                got = hs.plan.slice_update(mids[j])
                ok = ok and all(_eq(got[n], exp[n]) for n in exp)
        q.put((rank, bool(ok)))
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def test_sharded_hierarchy_gloo_world2():
    _run(_hier_worker)


def test_sharded_hierarchy_gloo_world3():
    _run(_hier_worker, world=3)


def test_plan_last_wave_quantum():
    """ShardPlan(last_wave_quantum=q): the last wave's per-rank size is the nearest whole
    multiple of q (>= 1), the other waves absorb the rest; coverage is unchanged; a quantum
    that does not fit (model too small, not a multiple of align) leaves the plan as is."""
    from flame_amd import shard
    G = 125_000_000
    model = {"model": torch.empty(G, dtype=torch.bfloat16, device="meta")}
    for world in (1, 2, 8):
        q = 2 * 256 * 2048
        p = shard.ShardPlan(model, world, 0, fracs=shard.HIER_FRACS, last_wave_quantum=q)
        waves = [sum(s.hi - s.lo for s in p.subs if s.wave == w and not s.tail) for w in range(p.n_waves)]
        assert p.n_waves == 2 and waves[-1] % q == 0 and waves[-1] >= q, waves
        ref = shard.ShardPlan(model, world, 0, fracs=shard.HIER_FRACS)
        assert abs(waves[-1] - sum(s.hi - s.lo for s in ref.subs if s.wave == 1)) <= q / 2 + 2048 * world
        assert p.owned_elements() == ref.owned_elements()
        for r in range(world):
            pr = shard.ShardPlan(model, world, r, fracs=shard.HIER_FRACS, last_wave_quantum=q)
            assert [(s.g0, s.g1) for s in pr.subs] == [(s.g0, s.g1) for s in p.subs]
        covered = sorted((s.g0 + r * ((s.g1 - s.g0) // world), s.g0 + (r + 1) * ((s.g1 - s.g0) // world))
                         for s in p.subs if not s.tail for r in range(world))
        assert covered[0][0] == 0 and all(a[1] == b[0] for a, b in zip(covered, covered[1:]))
    small = {"model": torch.empty(3 * 2048, dtype=torch.float32, device="meta")}
    a = shard.ShardPlan(small, 1, 0, fracs=shard.HIER_FRACS, last_wave_quantum=1 << 20)
    b = shard.ShardPlan(small, 1, 0, fracs=shard.HIER_FRACS)
    assert [(s.g0, s.g1) for s in a.subs] == [(s.g0, s.g1) for s in b.subs]
    odd = shard.ShardPlan(model, 2, 0, fracs=shard.HIER_FRACS, last_wave_quantum=1000)    # not a multiple of align
    assert [(s.g0, s.g1) for s in odd.subs] == [(s.g0, s.g1) for s in
                                                shard.ShardPlan(model, 2, 0, fracs=shard.HIER_FRACS).subs]


def test_sharded_paths_gloo_world8():
    """The N = 8 layout the driver's 8-GPU runs use (every rank owns 1/8 of each wave, the
    tails replicated), rehearsed with 8 gloo ranks on CPU: sharded FedAvg in waves, FedOPT +
    FedBuff and the sharded hierarchy, each bitwise against one process / the oracle."""
    _run(_fedavg_worker, world=8)
    _run(_opt_worker, world=8)
    _run(_hier_worker, world=8)


def _egress_worker(rank, world, port, q):
    """ShardedOptimizer(gather=False) + ShardedEgress: no all-gather; every rank writes only its
    ranges (rank 0 also the tails and the pickle's bytes) into one shared payload, which decodes --
    through the trainers' cloudpickle.loads -- to exactly the single-process FedAvg result."""
    dist = _init(rank, world, port)
    try:
        import cloudpickle
        from oracle import oracle as O
        import scenarios as S
        from flame_amd.egress import ShardedEgress
        g = torch.Generator().manual_seed(11)
        shapes = {k: v for k, v in FEDAVG_SHAPES.items() if k != "mask"}
        base = _model(g, shapes, 1.0)
        opt = shard.ShardedOptimizer(O.OracleFedAvg(), device=torch.device("cpu"), align=8, gather=False)
        eg = None
        ok = True
        before = sum(shard.GATHER_STATS.values())
        mine = {k: v.clone() for k, v in base.items()}
        ref = {k: v.clone() for k, v in base.items()}
        for r in range(3):
            n = 7
            clients = [_model(g, shapes, 1e-2) for _ in range(n)]
            counts = torch.randint(1, 1000, (n,), generator=g).tolist()
            ca, cb = S.SortedCache(), S.SortedCache()
            for i in range(n):
                ca[f"{i:02d}"] = S.TR({k: v.clone() for k, v in clients[i].items()}, counts[i])
                cb[f"{i:02d}"] = S.TR({k: v.clone() for k, v in clients[i].items()}, counts[i])
            out = opt.do(mine, ca, total=sum(counts))
            ok = ok and out is mine
            O.OracleFedAvg().do(ref, cb, total=sum(counts))
            if eg is None:
                eg = ShardedEgress(opt.plan, f"flametestegress{port}")
            payload = eg.encode({"weights": mine, "round": r})
            if rank == 0:
                msg = cloudpickle.loads(bytes(payload))
                ok = ok and msg["round"] == r and all(_eq(msg["weights"][k], ref[k]) for k in ref)
            else:
                ok = ok and payload is None
            # the model's non-owned ranges were never exchanged (rank-local state differs)
            if world > 1 and rank == 1:
                big = max(shapes, key=lambda k: torch.Size(shapes[k][0]).numel())
                ok = ok and not _eq(mine[big], ref[big])
        ok = ok and sum(shard.GATHER_STATS.values()) == before
        eg.close()
        q.put((rank, bool(ok)))
    except Exception as e:  # noqa: BLE001
        import traceback
        traceback.print_exc()
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_egress_without_gathers(world):
    _run(_egress_worker, world=world)


def _one(w):
    import scenarios as S
    c = S.SortedCache()
    c["a"] = S.TR({"w": w}, 3)
    return c


def test_gather_false_refuses_an_optimizer_that_does_not_write_in_place():
    """ShardedOptimizer(gather=False) leaves the model sharded in the caller's tensors, so the
    wrapped do() must write in place (FedAvg / FedProx); FedOPT's new current_weights refuse."""
    from oracle import oracle as O
    import scenarios as S
    g = torch.Generator().manual_seed(3)
    model = {"w": torch.randn(4096, generator=g)}
    opt = shard.ShardedOptimizer(O.OracleFedAvg(), device=torch.device("cpu"), align=8, gather=False)
    c = S.SortedCache()
    upd = torch.randn(4096, generator=g)
    c["a"] = S.TR({"w": upd.clone()}, 3)
    expect = O.OracleFedAvg().do({"w": model["w"].clone()}, _one(upd), total=3)
    out = opt.do(model, c, total=3)
    assert out is model
    assert torch.equal(out["w"], expect["w"])

    class NotInPlace:
        def do(self, base, cache, *, total=0, version=0, **kw):
            for k in list(cache.iterkeys()):
                cache.pop(k)
            return {k: v.clone() for k, v in base.items()}
    bad = shard.ShardedOptimizer(NotInPlace(), device=torch.device("cpu"), align=8, gather=False)
    c2 = S.SortedCache()
    c2["a"] = S.TR({"w": torch.randn(4096, generator=g)}, 3)
    with pytest.raises(NotImplementedError, match="in-place optimizer"):
        bad.do({"w": torch.randn(4096, generator=g)}, c2, total=3)
