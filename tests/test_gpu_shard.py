"""GPU parity of the parameter-sharded paths (flame_amd.shard) through the HIP kernels.

Two gloo ranks share the one MI355X of a test box (the driver's 8-GPU runs use RCCL):
each rank keeps only its slices of every update (``DeviceUpdateCache(shard=plan)``),
runs the HIP drop-ins on them wave by wave and all-gathers the model in place.  The
gathered model must equal one process's result bitwise, and the reference-generated
hierarchy fixture.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

import scenarios as S

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module", autouse=True)
def _native_loaded():
    from flame_amd import _native
    _native.lib()
    assert torch.cuda.is_available()


def _eq(a, b):
    a, b = a.detach().cpu(), b.detach().cpu()
    if a.dtype != b.dtype or a.shape != b.shape:
        return False
    if a.dtype in (torch.bfloat16, torch.float16):
        return torch.equal(a.view(torch.int16), b.view(torch.int16))
    return torch.equal(a, b)


def _two_ranks(target, world=2, timeout=150):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=target, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=timeout) for _ in ps)
    for p in ps:
        p.join(timeout=30)
    assert res == {r: True for r in range(world)}, res


def _init(rank, world, port):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)   # ranks share the one GPU
    return dist


def _model(g, P):
    return {"w": torch.randn(P, generator=g), "m": torch.randn(31, 129, generator=g),
            "bf": torch.randn(9001, generator=g).bfloat16(), "h": torch.randn(777, generator=g).half(),
            "d": torch.randn(2051, generator=g).double(), "nbt": torch.tensor(3, dtype=torch.int64),
            "z": torch.empty(0, 3)}


def _update(g, tmpl, i, scale=1e-2):
    def one(v):
        if v.is_floating_point():
            return (torch.randn(v.shape, generator=g) * scale).to(v.dtype)
        if v.dim() == 0:
            return torch.tensor(i, dtype=v.dtype)
        return torch.randint(0, 2 if v.dtype == torch.bool else 120, v.shape, generator=g).to(v.dtype)
    return {k: one(v) for k, v in tmpl.items()}


# ---------------------------------------------------------------- single process
def test_slabref_rows_equal_full_reduce():
    """Every rank's SlabRef slices of full-model slab slots (pointer rows from slot numbers)
    reduce to exactly the full reduction's elements, for every rank of a 3-way plan."""
    from flame_amd import engine, shard
    from flame_amd.slab import UpdateSlab
    g = torch.Generator().manual_seed(47)
    n, P = 9, 3 * 3 * 2048 * 5 + 333
    tmpl = {"a": torch.empty(P), "b": torch.empty(P // 2, dtype=torch.bfloat16), "c": torch.empty(7, 3)}
    slab = UpdateSlab(tmpl, capacity=16, device=DEV)
    ws = [slab.put({k: (torch.randn(v.shape, generator=g) * 1e-2).to(v.dtype).to(DEV) for k, v in tmpl.items()})
          for _ in range(n)]
    rates = [(i + 1) / 45 for i in range(n)]
    base = {k: torch.randn(v.shape, generator=g).to(v.dtype).to(DEV) for k, v in tmpl.items()}
    full = {k: v.clone() for k, v in base.items()}
    engine.accumulate(full, list(zip(ws, rates)))
    for rank in range(3):
        plan = shard.ShardPlan(tmpl, 3, rank)
        assert any(not s.tail for s in plan.subs) and any(s.tail for s in plan.subs)
        mine = {k: v.clone().reshape(-1) for k, v in base.items()}
        local = plan.views(mine)
        refs = [plan.local(w) for w in ws]
        assert all(type(r).__name__ == "SlabRef" for r in refs)
        assert engine.slab_rows(refs, plan.names, plan.local_numel, {n_: plan.dtypes[plan.by_name[n_].key]
                                                                      for n_ in plan.names}, torch.device(DEV))
        engine.accumulate(local, list(zip(refs, rates)))
        waved = {k: v.clone().reshape(-1) for k, v in base.items()}
        lw = plan.views(waved)
        for wave in range(plan.n_waves):     # restricted to one wave (one launch per dtype)
            engine.accumulate({n_: lw[n_] for n_ in plan.wave_names[wave]},
                              [(plan.restrict(r, wave), x) for r, x in zip(refs, rates)])
        torch.cuda.synchronize()
        for s in plan.subs:
            assert _eq(mine[s.key][s.lo:s.hi], full[s.key].reshape(-1)[s.lo:s.hi]), (rank, s.name)
            assert _eq(waved[s.key][s.lo:s.hi], full[s.key].reshape(-1)[s.lo:s.hi]), (rank, s.name)


# ---------------------------------------------------------------- FedAvg waves, two ranks
def _fedavg_narrow_worker(rank, world, port, q):
    _fedavg_worker(rank, world, port, q, narrow=True)


def _fedavg_overflow_worker(rank, world, port, q):
    _fedavg_worker(rank, world, port, q, capacity=4)


def _fedavg_worker(rank, world, port, q, narrow=False, capacity=16):
    dist = _init(rank, world, port)
    try:
        from flame_amd import engine, shard
        from flame_amd.ingest import DeviceUpdateCache
        from flame_amd.optimizers import optimizer_provider
        g = torch.Generator().manual_seed(51)
        tmpl = _model(g, 300_007)
        if narrow:   # a bool mask and a uint8 buffer, split across the ranks like any key
            tmpl["mask"] = torch.rand(40_961, generator=g) < 0.3
            tmpl["u8"] = torch.randint(0, 120, (8195,), generator=g).to(torch.uint8)
        opt = shard.ShardedOptimizer(optimizer_provider.get("fedavg"), device=torch.device(DEV))
        opt.set_layout(tmpl)
        cache = DeviceUpdateCache(device=DEV, placement="slab", capacity=capacity, shard=opt.plan)
        single = optimizer_provider.get("fedavg")
        ws = {k: v.to(DEV) for k, v in tmpl.items()}
        wr = {k: v.clone() for k, v in ws.items()}
        ok = opt.plan.n_waves == 3
        for r in range(3):
            ups = [_update(g, tmpl, 3 * r + i) for i in range(7)]
            counts = [11 + 7 * i for i in range(7)]
            cb = S.SortedCache()
            for i, u in enumerate(ups):
                cache[f"t{i}"] = S.TR(u, counts[i])        # host update: H2D of this rank's ranges only
                cb[f"t{i}"] = S.TR({k: v.to(DEV) for k, v in u.items()}, counts[i])
            mine = {k: v.clone() for k, v in ws.items()}
            engine.kernel_events = []
            out = opt.do(mine, cache, total=sum(counts), num_trainers=7)
            names = [e[0] for e in engine.kernel_events]
            engine.kernel_events = None
            ok = ok and out is mine and len(cache) == 0 and names.count("flame_agg_reduce") >= opt.plan.n_waves
            wr = single.do({k: v.clone() for k, v in wr.items()}, cb, total=sum(counts))
            torch.cuda.synchronize()
            ok = ok and all(_eq(out[k], wr[k]) for k in wr)
            ws = out
        q.put((rank, bool(ok)))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def test_sharded_fedavg_waves_two_ranks_one_gpu():
    """ShardedOptimizer(FedAvg) with rank-local slab caches: three waves, in-place gathers,
    bitwise == one process over 3 rounds (f32 / bf16 / f16 / f64 / int64 keys)."""
    _two_ranks(_fedavg_worker)


def test_sharded_fedavg_slab_overflow_two_ranks_one_gpu():
    """7 updates per round into a rank-local slab of 4 slots: the overflow stays one tensor
    per owned range (HBM) and the round mixes both layouts: == one process, bitwise."""
    _two_ranks(_fedavg_overflow_worker)


def test_sharded_fedavg_narrow_dtypes_two_ranks_one_gpu():
    """The same with a bool mask and a uint8 buffer in the model (their ranges stay one
    allocation per tensor in the rank's cache; torch's or / wrapping adds): == one process."""
    _two_ranks(_fedavg_narrow_worker)


# ---------------------------------------------------------------- config 5, two ranks
def _hier_fixture_worker(rank, world, port, q):
    dist = _init(rank, world, port)
    try:
        from fixture_io import Fixture
        from flame_amd import engine, shard
        from flame_amd.ingest import DeviceUpdateCache
        ok = True
        for name in S.HIER_FIXTURES:        # 2 x 3 bf16; 18 x 2 over f32 / f16 / bf16 (LDS groups)
            fx = Fixture(os.path.join(GOLD, name))
            rnd = fx.meta["round"]
            mids, arr, mver = S.hier_shape(fx.meta)
            top_w0 = S.to_dev(fx.weights("top_w0"), DEV)
            hier = shard.ShardedHierarchy(top_w0, align=8)
            ok = ok and hier.plan.n_waves == 2
            dc = DeviceUpdateCache(device=DEV, placement="slab", capacity=mids * arr, shard=hier.plan)
            middles = []
            for mid in range(mids):
                opt, agg = hier.middle_optimizer(), None
                for t in range(arr):
                    key = f"m{mid}t{t}"
                    dc[key] = S.TR(fx.weights(f"m{mid}/update{t}"), 10 + t, rnd - t % 2)
                    c = S.SortedCache()
                    c[key] = dc.pop(key)
                    agg = opt.do(agg, c, total=10 + t, version=rnd)
                middles.append(({k: v.clone() for k, v in top_w0.items()}, agg, arr, mver[mid]))
            top = {k: v.clone() for k, v in top_w0.items()}
            engine.kernel_events = []
            _, deltas = hier.round(middles, None, version=rnd, top_weights=top, top_goal=mids, with_delta=True)
            names = [e[0] for e in engine.kernel_events]
            engine.kernel_events = None
            # one pass per wave and dtype, no separate launches
            ok = ok and set(names) == {"flame_hier_fedbuff"} and len(names) >= hier.plan.n_waves
            torch.cuda.synchronize()
            ok = ok and all(_eq(top[k], fx.weights("top_out")[k]) for k in top)
            for mid in range(mids):
                exp = hier.plan.slice_update(fx.weights(f"m{mid}/delta"))
                ok = ok and all(_eq(deltas[mid][n], exp[n]) for n in exp)
        q.put((rank, bool(ok)))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def test_sharded_hierarchy_fixture_two_ranks_one_gpu():
    """ShardedHierarchy on the reference-generated hier_fedbuff_small fixture: every rank's
    top model == the reference's, bitwise; its middle deltas == its slices of the reference's."""
    _two_ranks(_hier_fixture_worker)


def _hier_random_worker(rank, world, port, q):
    dist = _init(rank, world, port)
    try:
        from flame_amd import shard
        from flame_amd.ingest import DeviceUpdateCache
        from flame_amd.optimizer.fedbuff import FedBuff, hierarchy_round
        from flame_amd.optimizer.sync_hierarchy import sync_hierarchy_round
        from flame_amd.slab import UpdateSlab
        g = torch.Generator().manual_seed(77)
        tmpl = {"w": torch.randn(300_007, generator=g).bfloat16(), "b": torch.randn(37, generator=g).bfloat16()}
        M, C, rnd = 3, 4, 9
        ups = [[_update(g, tmpl, 0) for _ in range(C)] for _ in range(M)]
        stale = [[(m + t) % 4 for t in range(C)] for m in range(M)]
        hier = shard.ShardedHierarchy(tmpl, device=torch.device(DEV))
        ok = hier.plan.n_waves == 2
        for own in (True, False):
            # sharded: rank-local slab caches
            dc = DeviceUpdateCache(device=DEV, placement="slab", capacity=M * C, shard=hier.plan)
            mids_s = []
            shared = {k: v.to(DEV) for k, v in tmpl.items()}
            for m in range(M):
                opt, agg = hier.middle_optimizer(), None
                for t in range(C):
                    key = f"m{m}t{t}"
                    dc[key] = S.TR(ups[m][t], 1, rnd - stale[m][t])
                    c = S.SortedCache()
                    c[key] = dc.pop(key)
                    agg = opt.do(agg, c, total=1, version=rnd)
                mids_s.append(({k: v.to(DEV) for k, v in tmpl.items()} if own else shared, agg, C, rnd - m % 2))
            top_s = {k: v.to(DEV) for k, v in tmpl.items()}
            agg_s, d_s = hier.round(mids_s, None, version=rnd, top_weights=top_s, top_goal=M, with_delta=True,
                                    update_middle_weights=own)
            # one process: full slab, one hierarchy_round
            slab = UpdateSlab(tmpl, capacity=M * C, device=DEV)
            mids_1 = []
            for m in range(M):
                opt, agg = FedBuff(), None
                for t in range(C):
                    c = S.SortedCache()
                    c[f"m{m}t{t}"] = S.TR(slab.put({k: v.to(DEV) for k, v in ups[m][t].items()}), 1,
                                          rnd - stale[m][t])
                    agg = opt.do(agg, c, total=1, version=rnd)
                mids_1.append(({k: v.to(DEV) for k, v in tmpl.items()}, agg, C, rnd - m % 2))
            top_1 = {k: v.to(DEV) for k, v in tmpl.items()}
            agg_1, d_1 = hierarchy_round(mids_1, None, version=rnd, top_weights=top_1, top_goal=M, with_delta=True,
                                         update_middle_weights=own)
            torch.cuda.synchronize()
            ok = ok and all(_eq(top_s[k], top_1[k]) for k in tmpl)
            exp_agg = hier.plan.slice_update(agg_1)
            ok = ok and all(_eq(agg_s[n], exp_agg[n]) for n in exp_agg)
            for m in range(M):
                exp = hier.plan.slice_update(d_1[m])
                ok = ok and all(_eq(d_s[m][n], exp[n]) for n in exp)
                if own:   # the middles' weights: this rank's ranges updated as one process does
                    got, want = hier.plan.slice_update(mids_s[m][0]), hier.plan.slice_update(mids_1[m][0])
                    ok = ok and all(_eq(got[n], want[n]) for n in want)
        # the synchronous hierarchy, same arrivals with sample counts
        counts = [[10 + 3 * m + t for t in range(C)] for m in range(M)]
        dc = DeviceUpdateCache(device=DEV, placement="slab", capacity=M * C, shard=hier.plan)
        specs_s, specs_1 = [], []
        slab = UpdateSlab(tmpl, capacity=M * C, device=DEV)
        for m in range(M):
            cs, c1 = S.SortedCache(), S.SortedCache()
            for t in range(C):
                dc[f"m{m}t{t}"] = S.TR(ups[m][t], counts[m][t])
                cs[f"m{m}t{t}"] = dc.pop(f"m{m}t{t}")
                c1[f"m{m}t{t}"] = S.TR(slab.put({k: v.to(DEV) for k, v in ups[m][t].items()}), counts[m][t])
            specs_s.append(({k: v.to(DEV) for k, v in tmpl.items()}, cs, sum(counts[m])))
            specs_1.append(({k: v.to(DEV) for k, v in tmpl.items()}, c1, sum(counts[m])))
        top_s = {k: v.to(DEV) for k, v in tmpl.items()}
        top_1 = {k: v.to(DEV) for k, v in tmpl.items()}
        hier.sync_round(specs_s, top_s)
        sync_hierarchy_round(specs_1, top_1)
        torch.cuda.synchronize()
        ok = ok and all(_eq(top_s[k], top_1[k]) for k in tmpl)
        for (ws, _, _), (w1, _, _) in zip(specs_s, specs_1):
            got, want = hier.plan.slice_update(ws), hier.plan.slice_update(w1)
            ok = ok and all(_eq(got[n], want[n]) for n in want)
        q.put((rank, bool(ok)))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def test_sharded_hierarchy_random_two_ranks_one_gpu():
    """ShardedHierarchy (async, own and fetched middle weights; and sync) with rank-local
    slab caches == one process's hierarchy_round / sync_hierarchy_round, bitwise: top model
    on every rank, each rank's slices of the top aggregate, deltas and middle weights."""
    _two_ranks(_hier_random_worker)


# ---------------------------------------------------------------- tiled middle weights
@pytest.mark.parametrize("mode", ["own", "fetched_rows", "sync", "fallback"])
def test_hierarchy_tiled_middles_equal_rows(mode):
    """Middle weights held as the slots of one tiled UpdateSlab (a chunk's middles are one
    block, flame_hier_segment.mid_tile_stride) == separate tensors, bitwise: middle weights,
    deltas, top aggregate and top weights; async FedBuff and sync FedAvg hierarchies, and the
    composed fallback (one middle's aggregate already flushed)."""
    from flame_amd.optimizer.fedbuff import FedBuff, hierarchy_round
    from flame_amd.optimizer.sync_hierarchy import sync_hierarchy_round
    from flame_amd.slab import UpdateSlab
    g = torch.Generator().manual_seed(91)
    tmpl = {"w": torch.randn(100_003, generator=g).bfloat16(), "b": torch.randn(37, generator=g).bfloat16(),
            "f": torch.randn(3000, generator=g)}
    M, C, rnd = 5, 3, 8
    ups = [[_update(g, tmpl, 0) for _ in range(C)] for _ in range(M)]
    store = UpdateSlab(tmpl, capacity=M * C, device=DEV)
    arrivals = [[store.put({k: v.to(DEV) for k, v in u.items()}) for u in row] for row in ups]
    mstore = UpdateSlab(tmpl, capacity=M, device=DEV)
    starts = [{k: (v + 0.5 * m).to(v.dtype) for k, v in tmpl.items()} for m in range(M)]
    res = {}
    for lay in ("rows", "tiled"):
        if lay == "rows":
            mids = [{k: v.to(DEV) for k, v in st.items()} for st in starts]
        else:
            mids = [mstore.put({k: v.to(DEV) for k, v in st.items()}) for st in starts]
        top = {k: v.to(DEV) for k, v in tmpl.items()}
        if mode == "sync":
            specs = []
            for m in range(M):
                c = S.SortedCache()
                for t in range(C):
                    c[f"{m}{t}"] = S.TR(arrivals[m][t], 10 + m + t)
                specs.append((mids[m], c, sum(10 + m + t for t in range(C))))
            _, deltas = sync_hierarchy_round(specs, top, with_delta=True)
            agg = None
        else:
            aggs = []
            for m in range(M):
                opt, a = FedBuff(), None
                for t in range(C):
                    c = S.SortedCache()
                    c[f"{m}{t}"] = S.TR(arrivals[m][t], 1, rnd - (m + t) % 3)
                    a = opt.do(a, c, total=1, version=rnd)
                aggs.append(a)
            if mode == "fallback":
                aggs[2].flush()
            agg, deltas = hierarchy_round([(mids[m], aggs[m], C, rnd - m % 2) for m in range(M)], None, version=rnd,
                                          top_weights=top, top_goal=M, with_delta=True,
                                          update_middle_weights=(mode != "fetched_rows"))
        torch.cuda.synchronize()
        res[lay] = ({k: v.cpu() for k, v in top.items()}, [S.to_cpu(d) for d in deltas],
                    None if agg is None else S.to_cpu(agg),
                    [{k: (mstore.read(w.slot, k) if lay == "tiled" else w[k]).cpu() for k in tmpl} for w in mids])
    a, b = res["rows"], res["tiled"]
    S.assert_bitwise("top", a[0], b[0])
    for m in range(M):
        S.assert_bitwise(f"delta{m}", a[1][m], b[1][m])
        S.assert_bitwise(f"mid{m}", a[3][m], b[3][m])
    if a[2] is not None:
        S.assert_bitwise("top agg", a[2], b[2])


# ---------------------------------------------------------------- the RCCL code path
def _rccl_world1_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    try:
        from flame_amd import engine, shard
        from flame_amd.ingest import DeviceUpdateCache
        from flame_amd.optimizers import optimizer_provider
        g = torch.Generator().manual_seed(57)
        # several large keys: every wave holds pieces of more than one key -> one coalesced
        # group of in-place all-gathers per wave (RCCL's allgather_into_tensor_coalesced)
        tmpl = {"a": torch.randn(300_001, generator=g), "b": torch.randn(200_003, generator=g),
                "c": torch.randn(150_000, generator=g).bfloat16(), "d": torch.randn(99_999, generator=g)}
        opt = shard.ShardedOptimizer(optimizer_provider.get("fedavg"), device=torch.device(DEV), align=1024)
        opt.set_layout(tmpl)
        multi = [w for w in range(opt.plan.n_waves)
                 if len({opt.plan.by_name[n].key for n in opt.plan.wave_names[w] if not opt.plan.by_name[n].tail}) > 1]
        ok = bool(multi)
        cache = DeviceUpdateCache(device=DEV, placement="slab", capacity=8, shard=opt.plan)
        single = optimizer_provider.get("fedavg")
        ws = {k: v.to(DEV) for k, v in tmpl.items()}
        wr = {k: v.clone() for k, v in ws.items()}
        for r in range(2):
            ups = [_update(g, tmpl, i) for i in range(5)]
            cb = S.SortedCache()
            for i, u in enumerate(ups):
                cache[f"t{i}"] = S.TR(u, 3 + i)
                cb[f"t{i}"] = S.TR({k: v.to(DEV) for k, v in u.items()}, 3 + i)
            ws = opt.do(ws, cache, total=25)
            wr = single.do(wr, cb, total=25)
            torch.cuda.synchronize()
            ok = ok and all(_eq(ws[k], wr[k]) for k in tmpl)
        # FedAdam: current_weights gathered into new tensors through the same coalesced path
        fa = shard.ShardedOptimizer(optimizer_provider.get("fedadam", beta_1=0.9, beta_2=0.99, eta=1e-2, tau=1e-3),
                                    device=torch.device(DEV), align=1024)
        fb = optimizer_provider.get("fedadam", beta_1=0.9, beta_2=0.99, eta=1e-2, tau=1e-3)
        wa, wb = {k: v.clone() for k, v in ws.items()}, {k: v.clone() for k, v in ws.items()}
        for r in range(3):
            ups = [_update(g, tmpl, i) for i in range(4)]
            ca, cb = S.SortedCache(), S.SortedCache()
            for i, u in enumerate(ups):
                ca[f"t{i}"] = S.TR({k: v.to(DEV) for k, v in u.items()}, 2 + i)
                cb[f"t{i}"] = S.TR({k: v.to(DEV) for k, v in u.items()}, 2 + i)
            wa = fa.do({k: v.clone() for k, v in wa.items()}, ca, total=14)
            wb = fb.do({k: v.clone() for k, v in wb.items()}, cb, total=14)
            torch.cuda.synchronize()
            ok = ok and all(_eq(wa[k], wb[k]) for k in tmpl)
        q.put((rank, bool(ok)))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def test_sharded_rccl_world1_coalesced_inplace_gathers():
    """The product's RCCL path (backend nccl = RCCL) as a world-1 group: in-place
    all_gather_into_tensor, coalesced across the keys of a wave, for FedAvg (into the
    caller's tensors) and FedAdam (into new tensors) == one process, bitwise."""
    _two_ranks(_rccl_world1_worker, world=1)


def _resnetish(g):
    """A ResNet-like state_dict: many keys of mixed sizes, BatchNorm buffers incl. int64."""
    out = {}
    shapes = [(64, 3, 7, 7)] + [(64, 64, 3, 3)] * 4 + [(128, 64, 3, 3), (128, 128, 3, 3), (128, 64, 1, 1)] + \
        [(256, 128, 3, 3), (256, 256, 3, 3)] + [(1000, 256), (1000,)]
    for i, s in enumerate(shapes):
        out[f"layer{i}.weight"] = torch.randn(s, generator=g)
        if len(s) == 4:
            c = s[0]
            out[f"bn{i}.weight"] = torch.randn(c, generator=g)
            out[f"bn{i}.bias"] = torch.randn(c, generator=g)
            out[f"bn{i}.running_mean"] = torch.randn(c, generator=g)
            out[f"bn{i}.running_var"] = torch.rand(c, generator=g)
            out[f"bn{i}.num_batches_tracked"] = torch.tensor(7, dtype=torch.int64)
    return out


def _many_keys_worker(rank, world, port, q):
    dist = _init(rank, world, port)
    try:
        from flame_amd import shard
        from flame_amd.ingest import DeviceUpdateCache
        from flame_amd.optimizers import optimizer_provider
        g = torch.Generator().manual_seed(81)
        tmpl = _resnetish(g)
        ok = len(tmpl) > 50
        for sort in ("fedavg", "fedadam"):
            kw = dict(beta_1=0.9, beta_2=0.99, eta=1e-2, tau=1e-3) if sort == "fedadam" else {}
            opt = shard.ShardedOptimizer(optimizer_provider.get(sort, **kw), device=torch.device(DEV))
            opt.set_layout(tmpl)
            ok = ok and sum(1 for s in opt.plan.subs if not s.tail) > 0
            cache = DeviceUpdateCache(device=DEV, placement="slab", capacity=8, shard=opt.plan)
            single = optimizer_provider.get(sort, **kw)
            ws = {k: v.to(DEV) for k, v in tmpl.items()}
            wr = {k: v.clone() for k, v in ws.items()}
            for r in range(3):
                ups = [_update(g, tmpl, 10 * r + i) for i in range(6)]
                cb = S.SortedCache()
                for i, u in enumerate(ups):
                    cache[f"t{i}"] = S.TR(u, 5 + i)
                    cb[f"t{i}"] = S.TR({k: v.to(DEV) for k, v in u.items()}, 5 + i)
                ws = opt.do({k: v.clone() for k, v in ws.items()}, cache, total=45)
                wr = single.do({k: v.clone() for k, v in wr.items()}, cb, total=45)
                torch.cuda.synchronize()
                ok = ok and list(ws) == list(wr) and all(_eq(ws[k], wr[k]) for k in tmpl)
        q.put((rank, bool(ok)))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def test_sharded_many_keys_resnet_like_two_ranks_one_gpu():
    """A ResNet-like state_dict (62 keys: conv / fc weights, BatchNorm affine + running stats +
    int64 num_batches_tracked) through ShardedOptimizer(FedAvg) and (FedAdam, which promotes
    the int64 buffers) with rank-local slab caches: == one process, bitwise, 3 rounds."""
    _two_ranks(_many_keys_worker)


def test_hier_wave_quantum_world1():
    """ShardedHierarchy(middles=M) on the GPU: the library's residency for the hierarchy
    launch (2 workgroups per CU with LDS-held store groups, more without) sizes the last
    wave to whole rounds of resident workgroups; the sharded round stays bitwise equal to
    one hierarchy_round (world 1, no process group) -- half of its middles taking their
    arrivals through ShardedOptimizer.do_arrivals."""
    from flame_amd import engine, shard
    from flame_amd.optimizer.fedbuff import FedBuff, hierarchy_round
    from flame_amd.slab import UpdateSlab
    big = engine.hier_resident_per_cu(engine.N.FLAME_BF16, 64)
    small = engine.hier_resident_per_cu(engine.N.FLAME_BF16, 2)
    assert big >= 1 and small >= big, (big, small)
    assert engine.hier_resident_per_cu(engine.N.FLAME_BF16, 64, sync=True) >= 1
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    M, C, rnd = 16, 2, 7
    q = engine.hier_resident_per_cu(engine.N.FLAME_BF16, M) * cus * engine.chunk_elems(engine.N.FLAME_BF16)
    P = 2 * q + 12_345
    g = torch.Generator().manual_seed(5)
    tmpl = {"w": torch.randn(P, generator=g).bfloat16(), "b": torch.randn(9, generator=g).bfloat16()}
    hier = shard.ShardedHierarchy(tmpl, device=torch.device(DEV), middles=M)
    waves = [sum(s.hi - s.lo for s in hier.plan.subs if s.wave == w and not s.tail) for w in range(hier.plan.n_waves)]
    assert hier.plan.n_waves == 2 and waves[-1] % q == 0, (waves, q)
    ups = [[{k: (torch.randn(v.shape, generator=g) * 1e-2).bfloat16() for k, v in tmpl.items()} for _ in range(C)]
           for _ in range(M)]
    outs = []
    for sharded in (True, False):
        slab = UpdateSlab(tmpl, capacity=M * C, device=DEV)
        mids = []
        for m in range(M):
            opt, agg = (hier.middle_optimizer() if sharded else FedBuff()), None
            if sharded and m % 2 == 0:     # the batched arrival API on half of the sharded middles
                agg = opt.do_arrivals(None, [S.TR(slab.put({k: v.to(DEV) for k, v in ups[m][t].items()}), 1,
                                                  rnd - (m + t) % 3) for t in range(C)], version=rnd)
            for t in range(C if agg is None else 0):
                c = S.SortedCache()
                c[f"m{m}t{t}"] = S.TR(slab.put({k: v.to(DEV) for k, v in ups[m][t].items()}), 1, rnd - (m + t) % 3)
                agg = opt.do(agg, c, total=1, version=rnd)
            mids.append(({k: v.to(DEV) for k, v in tmpl.items()}, agg, C, rnd - m % 2))
        top = {k: v.to(DEV) for k, v in tmpl.items()}
        if sharded:
            hier.round(mids, None, version=rnd, top_weights=top, top_goal=M)
        else:
            hierarchy_round(mids, None, version=rnd, top_weights=top, top_goal=M)
        torch.cuda.synchronize()
        outs.append((top, [m[0] for m in mids]))
    for k in tmpl:
        assert _eq(outs[0][0][k], outs[1][0][k]), k
        for a, b in zip(outs[0][1], outs[1][1]):
            assert _eq(a[k], b[k]), k


def test_sharded_fedbuff_scale_add_waves_world1():
    """The async top sharded (ShardedOptimizer(FedBuff, accumulate_only=True)): arrivals one
    per do() on this rank's slices, then scale_add_agg_weights -- one fused launch per wave
    in place (the waves' gathers behind them) -- bitwise equal to the unsharded FedBuff, for
    fused and unfused scale_add and a multi-key, mixed-dtype model."""
    from flame_amd import shard
    from flame_amd.optimizer.fedbuff import FedBuff
    g = torch.Generator().manual_seed(31)
    tmpl = {"w": torch.randn(700_001, generator=g), "h": torch.randn(3001, 17, generator=g).bfloat16(),
            "b": torch.randn(5, generator=g)}
    K, rnd = 7, 9
    ups = [{k: (torch.randn(v.shape, generator=g) * 1e-2).to(v.dtype) for k, v in tmpl.items()} for _ in range(K)]
    for fuse in (True, False):
        outs = []
        for sharded in (True, False):
            inner = FedBuff(fuse_scale_add=fuse)
            opt = shard.ShardedOptimizer(inner, device=torch.device(DEV), accumulate_only=True) if sharded else inner
            model = {k: v.to(DEV) for k, v in tmpl.items()}
            if sharded:
                opt.set_layout(model)
                assert opt.plan.n_waves == 3
            agg = None
            for i in range(K):
                c = S.SortedCache()
                c[f"{i:02d}"] = S.TR({k: v.to(DEV) for k, v in ups[i].items()}, 1, rnd - i % 3)
                agg = opt.do(agg, c, total=1, version=rnd)
            out = opt.scale_add_agg_weights(model, agg, K)
            torch.cuda.synchronize()
            assert out is model
            outs.append(model)
        for k in tmpl:
            assert _eq(outs[0][k], outs[1][k]), (fuse, k)


# ---------------------------------------------------------------- sharded egress, two ranks
def _egress_worker(rank, world, port, q):
    """ShardedOptimizer(gather=False) on the HIP FedAvg + ShardedEgress: updates arrive as decoded
    channel payloads (views at arbitrary alignment) into DeviceUpdateCache(shard=plan); no gather
    runs; every rank D2Hs its ranges into the one shared, registered egress segment; rank 0's
    payload decodes (cloudpickle.loads) to one process's FedAvg result, bitwise, over two rounds."""
    dist = _init(rank, world, port)
    try:
        import cloudpickle
        from flame_amd import ingest, shard
        from flame_amd.egress import ShardedEgress
        from flame_amd.ingest import DeviceUpdateCache
        from flame_amd.optimizers import optimizer_provider
        g = torch.Generator().manual_seed(61)
        tmpl = _model(g, 300_007)
        del tmpl["z"]
        opt = shard.ShardedOptimizer(optimizer_provider.get("fedavg"), device=torch.device(DEV), gather=False)
        opt.set_layout(tmpl)
        cache = DeviceUpdateCache(device=DEV, placement="slab", capacity=8, shard=opt.plan)
        mine = {k: v.clone().to(DEV) for k, v in tmpl.items()}
        ref = {k: v.clone().to(DEV) for k, v in tmpl.items()}
        single = optimizer_provider.get("fedavg")
        eg = ShardedEgress(opt.plan, f"flamegpuegress{port}")
        before = sum(shard.GATHER_STATS.values())
        ok = True
        for r in range(2):
            n = 5
            ups = [_update(g, tmpl, i) for i in range(n)]
            counts = [10 + 7 * i for i in range(n)]
            payloads = [cloudpickle.dumps({"weights": u, "dataset_size": c}) for u, c in zip(ups, counts)]
            rc = S.SortedCache()
            for i, b in enumerate(payloads):
                msg = ingest.decode(b)
                cache[f"{i:02d}"] = S.TR(msg["weights"], msg["dataset_size"])
                rc[f"{i:02d}"] = S.TR({k: v.to(DEV) for k, v in ups[i].items()}, counts[i])
            out = opt.do(mine, cache, total=sum(counts))
            ok = ok and out is mine
            single.do(ref, rc, total=sum(counts))
            payload = eg.encode({"weights": mine, "round": r})
            if rank == 0:
                got = cloudpickle.loads(bytes(payload))
                ok = ok and got["round"] == r and all(_eq(got["weights"][k], ref[k]) for k in ref)
            else:
                ok = ok and payload is None
        ok = ok and sum(shard.GATHER_STATS.values()) == before
        eg.close()
        q.put((rank, bool(ok)))
    except Exception as e:  # noqa: BLE001
        import traceback
        traceback.print_exc()
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def test_sharded_egress_two_ranks_one_gpu():
    _two_ranks(_egress_worker)
