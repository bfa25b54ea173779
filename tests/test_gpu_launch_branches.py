"""Launch branches that only long launches reach, each pinned to the oracle bitwise.

flame_hier_fedbuff's one-middle low-residency instantiation (kHLo*: one middle, >= 64
arrivals, >= 4,096 chunks, FedBuff mode) is what the async FedBuff top's fused
scale_add (asyncfl/top_aggregator.py:85-110, optimizer/fedbuff.py:101-127) and a lone
middle's scale_add + upload delta (asyncfl/middle_aggregator.py:221-226,246) run at
aggGoal >= 64.  Its client unroll is 3, so arrival counts 64, 65 and 67 run every tail
of the unrolled loop.  Both entry points are covered: the kernel-argument launch (a model
of a few keys, the common case) and the device-table launch (engine.ARGMETA off, as a
many-key model takes it).  Every case asserts, through the C ABI's launch-branch
counters, that the launch took the branch it is meant to pin.

Also here: FedOPT at >= 8,192 chunks in bf16 / f16 (one chunk per workgroup: the
multi-chunk grid is fp32-only), and the eager caller's aliased FedOPT step
(FLAME_SEG_CUR_IS_AVG) through the fused kernel.
"""

import pytest
import torch

import scenarios as S

pytestmark = [pytest.mark.gpu, pytest.mark.oracle]

DEV = "cuda:0"
RND = 20
DTS = {"f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16}


def _oracle():
    from oracle import oracle as O
    return O


def _counts():
    from flame_amd import _native
    return _native.launch_branch_counts()


def _diff(before, after):
    return {k: after[k] - before.get(k, 0) for k in after if after[k] != before.get(k, 0)}


def _shapes(dtype):
    from flame_amd import engine
    chunk = engine.chunk_elems(engine.dtype_code(dtype))
    return [("w", 4096 * chunk), ("t", 4_099)]          # >= 4,096 chunks + a ragged key


_DATA = {}


def _arrivals(dtype, n):
    """n synthetic arrivals (device, CPU copies) and a base model; cached per dtype."""
    from flame_amd import engine
    key = dtype
    if key not in _DATA or len(_DATA[key][0]) < n:
        _DATA.clear()
        shapes = _shapes(dtype)
        dev_w, cpu_w = [], []
        for i in range(67):
            w = {}
            for j, (k, s) in enumerate(shapes):
                t = torch.empty(s, dtype=dtype, device=DEV)
                engine.synth_fill_(t, 31, 100 + 2 * i + j, 0, 1e-2)
                w[k] = t
            dev_w.append(w)
            cpu_w.append({k: v.cpu() for k, v in w.items()})
        base = {}
        for j, (k, s) in enumerate(shapes):
            t = torch.empty(s, dtype=dtype, device=DEV)
            engine.synth_fill_(t, 31, j, 0, 1.0)
            base[k] = t
        _DATA[key] = (dev_w, cpu_w, base)
    dev_w, cpu_w, base = _DATA[key]
    return dev_w[:n], cpu_w[:n], base


def _versions(n):
    return [RND - (i * 3) % 5 for i in range(n)]


_ORACLE_AGGS = {}


def _oracle_agg(cpu_w, vers, start=None):
    """OracleFedBuff over the arrivals (one do() each); None-start results are cached per
    (dtype, arrival count): the cases share the synthetic arrivals.  Read-only for callers."""
    key = (cpu_w[0]["w"].dtype, len(cpu_w), tuple(vers)) if start is None else None
    if key is not None and key in _ORACLE_AGGS:
        return _ORACLE_AGGS[key]
    agg = _oracle_agg_compute(cpu_w, vers, start)
    if key is not None:
        if any(k[0] != key[0] for k in _ORACLE_AGGS):
            _ORACLE_AGGS.clear()      # one dtype's worth at a time (host memory)
        _ORACLE_AGGS[key] = agg
    return agg


def _oracle_agg_compute(cpu_w, vers, start=None):
    O = _oracle()
    ora = O.OracleFedBuff()
    agg = {k: v.clone() for k, v in start.items()} if start is not None else None
    for i, w in enumerate(cpu_w):
        c = S.SortedCache()
        c[f"{i:03d}"] = S.TR({k: v.clone() for k, v in w.items()}, 1, vers[i])
        agg = ora.do(agg, c, total=1, version=RND)
    return agg


CASES = [(dt, placement, with_delta, path)
         for dt in DTS for placement in ("slab", "tensors") for with_delta in (False, True)
         for path in ("argmeta", "table")]


@pytest.mark.parametrize("dt,placement,with_delta,path", CASES,
                         ids=["-".join(map(str, c)) for c in CASES])
def test_fedbuff_fused_scale_add_low_residency_vs_oracle(dt, placement, with_delta, path, monkeypatch):
    """The async top's round at aggGoal 64 / 65 / 67 (one do() per arrival, None start), then
    scale_add (+ the middle's delta) fused from the queued arrivals: ONE low-residency
    flame_hier_fedbuff launch, every element bitwise == OracleFedBuff per arrival +
    scale_add_tensor(want_delta=True)."""
    from flame_amd import engine
    from flame_amd.slab import UpdateSlab
    O = _oracle()
    dtype = DTS[dt]
    n = (64, 65, 67)[CASES.index((dt, placement, with_delta, path)) % 3]
    dev_w, cpu_w, base = _arrivals(dtype, n)
    vers = _versions(n)
    if path == "table":
        monkeypatch.setattr(engine, "ARGMETA", False)
    slab = None
    if placement == "slab":
        slab = UpdateSlab({k: torch.empty(v.shape, dtype=dtype) for k, v in base.items()}, capacity=n,
                          device=DEV)
    opt = S_make("fedbuff")
    agg = None
    for i in range(n):
        c = S.SortedCache()
        c[f"{i:03d}"] = S.TR(slab.put(dev_w[i]) if slab is not None else dev_w[i], 1, vers[i])
        agg = opt.do(agg, c, total=1, version=RND)
    w = {k: v.clone() for k, v in base.items()}
    before = _counts()
    if with_delta:
        _, delta = opt.scale_add_agg_weights_with_delta(w, agg, n)
    else:
        opt.scale_add_agg_weights(w, agg, n)
    torch.cuda.synchronize()
    hits = _diff(before, _counts())
    want = f"flame_hier_fedbuff{'_argmeta' if path == 'argmeta' else ''}/lo/{dt}/fedbuff"
    assert hits == {want: 1}, hits
    exp_agg = _oracle_agg(cpu_w, vers)
    wo = {k: v.cpu() for k, v in base.items()}
    do_ = {k: O.scale_add_tensor(wo[k], exp_agg[k], n, want_delta=True) for k in wo}
    S.assert_bitwise(f"lo/{dt}/{placement}/{path}/n{n}/w", S.to_cpu(w), wo)
    if with_delta:
        S.assert_bitwise(f"lo/{dt}/{placement}/{path}/n{n}/delta", S.to_cpu(delta), do_)
    # the aggregate stays readable: its queued arrivals are reduced on this read
    S.assert_bitwise(f"lo/{dt}/{placement}/{path}/n{n}/agg", S.to_cpu(dict(agg)), exp_agg)
    del slab, agg


def S_make(sort, **kw):
    from flame_amd.optimizers import optimizer_provider
    return optimizer_provider.get(sort, **kw)


@pytest.mark.parametrize("dt", list(DTS))
def test_fedbuff_existing_aggregate_long_round_vs_oracle(dt):
    """An existing aggregate (a dict the caller passes in, fedbuff.py:157) + a round of 65
    arrivals in one do_arrivals call: one low-residency flame_agg_reduce launch (accumulate,
    not init-first); the fused scale_add does not apply to a materialised aggregate, so the
    scale_add + delta is its own launch -- both bitwise == the oracle."""
    O = _oracle()
    dtype = DTS[dt]
    n = 65
    dev_w, cpu_w, base = _arrivals(dtype, n)
    vers = _versions(n)
    g = torch.Generator().manual_seed(5)
    prev = {k: (torch.randn(v.shape, generator=g) * 1e-3).to(dtype) for k, v in base.items()}
    opt = S_make("fedbuff")
    before = _counts()
    agg = opt.do_arrivals({k: v.to(DEV) for k, v in prev.items()}, [S.TR(dev_w[i], 1, vers[i]) for i in range(n)],
                          version=RND)
    torch.cuda.synchronize()
    hits = _diff(before, _counts())
    assert hits == {f"flame_agg_reduce_argmeta/lo_burst/{dt}": 1}, hits
    w = {k: v.clone() for k, v in base.items()}
    before = _counts()
    _, delta = opt.scale_add_agg_weights_with_delta(w, agg, n)
    torch.cuda.synchronize()
    hits = _diff(before, _counts())
    assert "flame_hier_fedbuff/lo" not in " ".join(hits), hits
    assert hits.get(f"flame_fedbuff_scale_add/{dt}") == 1, hits
    exp_agg = _oracle_agg(cpu_w, vers, start=prev)
    S.assert_bitwise(f"existing/{dt}/agg", S.to_cpu(agg), exp_agg)
    wo = {k: v.cpu() for k, v in base.items()}
    do_ = {k: O.scale_add_tensor(wo[k], exp_agg[k], n, want_delta=True) for k in wo}
    S.assert_bitwise(f"existing/{dt}/w", S.to_cpu(w), wo)
    S.assert_bitwise(f"existing/{dt}/delta", S.to_cpu(delta), do_)


HIER_CASES = [(dt, path, readonly) for dt in DTS for path in ("argmeta", "table") for readonly in (False, True)]


@pytest.mark.parametrize("dt,path,readonly", HIER_CASES, ids=["-".join(map(str, c)) for c in HIER_CASES])
def test_lone_middle_hierarchy_round_low_residency_vs_oracle(dt, path, readonly, monkeypatch):
    """A lone middle (67 queued arrivals) feeding an EXISTING top aggregate and applying the
    top's scale_add, in one hierarchy_round: the low-residency launch with TOP_ACCUM and
    TOP_APPLY (and MID_READONLY), bitwise == the roles' op sequence on the oracle: the
    middle's FedBuff + scale_add + delta (asyncfl/middle_aggregator.py:221-226,246), the top's
    FedBuff.do of the delta (asyncfl/top_aggregator.py:85-92) and scale_add (:104-110)."""
    from flame_amd import engine
    from flame_amd.optimizer.fedbuff import hierarchy_round
    O = _oracle()
    dtype = DTS[dt]
    n = 67
    dev_w, cpu_w, base = _arrivals(dtype, n)
    vers = _versions(n)
    if path == "table":
        monkeypatch.setattr(engine, "ARGMETA", False)
    g = torch.Generator().manual_seed(9)
    top_prev = {k: (torch.randn(v.shape, generator=g) * 1e-3).to(dtype) for k, v in base.items()}
    top_w0 = {k: torch.randn(v.shape, generator=g).to(dtype) for k, v in base.items()}
    opt = S_make("fedbuff")
    agg = opt.do_arrivals(None, [S.TR(dev_w[i], 1, vers[i]) for i in range(n)], version=RND)
    mid = {k: v.clone() for k, v in base.items()}
    top_agg = {k: v.to(DEV) for k, v in top_prev.items()}
    top_w = {k: v.to(DEV) for k, v in top_w0.items()}
    mver = RND - 2
    before = _counts()
    _, deltas = hierarchy_round([(mid, agg, n, mver)], top_agg, version=RND, top_weights=top_w, top_goal=3,
                                with_delta=True, update_middle_weights=not readonly)
    torch.cuda.synchronize()
    hits = _diff(before, _counts())
    want = f"flame_hier_fedbuff{'_argmeta' if path == 'argmeta' else ''}/lo/{dt}/fedbuff"
    assert hits == {want: 1}, hits
    # the oracle: the roles' separate calls
    exp_agg = _oracle_agg(cpu_w, vers)
    mo = {k: v.cpu() for k, v in base.items()}
    do_ = {k: O.scale_add_tensor(mo[k], exp_agg[k], n, want_delta=True) for k in mo}
    ora_top = O.OracleFedBuff()
    c = S.SortedCache()
    c["mid"] = S.TR({k: v.clone() for k, v in do_.items()}, 1, mver)
    tao = ora_top.do({k: v.clone() for k, v in top_prev.items()}, c, total=1, version=RND)
    two = {k: v.clone() for k, v in top_w0.items()}
    ora_top.scale_add_agg_weights(two, tao, 3)
    S.assert_bitwise(f"hier-lo/{dt}/{path}/delta", S.to_cpu(deltas[0]), do_)
    S.assert_bitwise(f"hier-lo/{dt}/{path}/top_agg", S.to_cpu(top_agg), tao)
    S.assert_bitwise(f"hier-lo/{dt}/{path}/top_w", S.to_cpu(top_w), two)
    S.assert_bitwise(f"hier-lo/{dt}/{path}/mid", S.to_cpu(mid), {k: v.cpu() for k, v in base.items()} if readonly else mo)


@pytest.mark.parametrize("dt", ["f32", "bf16", "f16"])
@pytest.mark.parametrize("sort", ["fedadam", "fedyogi", "fedadagrad"])
@pytest.mark.parametrize("path", ["argmeta", "table"])
def test_fedopt_long_launch_every_entry_point(dt, sort, path, monkeypatch):
    """FedOPT over >= 8,192 chunks through both entry points: fp32 takes the multi-chunk
    (LDS-held outputs) instantiation, bf16 / f16 one chunk per workgroup over the whole grid
    (the round-3 device-table launch sized the grid for the multi-chunk fp32 kernel and left
    3/4 of a bf16 / f16 model unreduced).  Every element, within the §8(c) contract against
    the reference's op sequence on the oracle's FedAvg (avg bitwise)."""
    O = _oracle()
    from flame_amd import engine
    if path == "table":
        monkeypatch.setattr(engine, "ARGMETA", False)
    dtype = DTS[dt]
    chunk = engine.chunk_elems(engine.dtype_code(dtype))
    P = 8 * 256 * 4 * chunk + 777
    n = 5
    cl = [torch.empty(P, dtype=dtype, device=DEV) for _ in range(n)]
    for i, t in enumerate(cl):
        engine.synth_fill_(t, 41, 1 + i, 0, 1e-2)
    cur0 = torch.empty(P, dtype=dtype, device=DEV)
    engine.synth_fill_(cur0, 41, 0, 0, 1.0)
    counts = [3, 1, 4, 1, 5]
    total = sum(counts)
    opt = S_make(sort)
    ora = O.OracleFedOPT(sort)
    got_cur = exp_cur = None
    for r in range(3):
        cache, ocache = S.SortedCache(), S.SortedCache()
        for i in range(n):
            cache[f"{i}"] = S.TR({"x": cl[(i + r) % n]}, counts[i])
            ocache[f"{i}"] = S.TR({"x": cl[(i + r) % n].cpu()}, counts[i])
        b = {"x": cur0.clone()} if got_cur is None else {"x": got_cur["x"].clone()}
        ob = {"x": cur0.cpu()} if exp_cur is None else {"x": exp_cur["x"].clone()}
        before = _counts()
        got_cur = opt.do(b, cache, total=total)
        exp_cur = ora.do(ob, ocache, total=total)
        torch.cuda.synchronize()
        if r >= 1:
            hits = _diff(before, _counts())
            entry = "flame_fedopt_reduce_adapt" + ("_argmeta" if path == "argmeta" else "")
            mode = f"multi/{dt}" if dt == "f32" else dt
            assert hits == {f"{entry}/{mode}/{sort}": 1}, hits
            S.assert_bitwise(f"{sort}/{dt}/r{r}/avg", S.to_cpu(opt.agg_weights), ora.agg_weights)
            if r == 1:      # round 1's step from identical state: elementwise contract
                S.assert_close_fedopt(f"{sort}/{dt}/r{r}/cur", S.to_cpu(got_cur), exp_cur)
            else:
                S.assert_close_fedopt(f"{sort}/{dt}/r{r}/cur", S.to_cpu(got_cur), exp_cur, elementwise=False)


@pytest.mark.parametrize("dt", list(DTS))
@pytest.mark.parametrize("sort", ["fedadam", "fedyogi", "fedadagrad"])
def test_fedopt_eager_aliased_step_fused(dt, sort):
    """The eager top aggregator's FedOPT round (eager_syncfl/top_aggregator.py:36-90): the
    same base dict goes to every do(), so after the round-1 passthrough current_weights IS
    base and the reference's d = avg - current is 0.  That step now runs in the fused kernel
    (FLAME_SEG_CUR_IS_AVG) -- one flame_fedopt_reduce_adapt launch, no torch op passes --
    and equals the reference op sequence on the oracle bitwise (m = v = 0 make every op exact)."""
    O = _oracle()
    dtype = DTS[dt]
    g = torch.Generator().manual_seed(17)
    shapes = {"a": (1000, 37), "b": (4099,)}
    base0 = {k: torch.randn(s, generator=g).to(dtype) for k, s in shapes.items()}
    ups = [{k: (torch.randn(s, generator=g) * 1e-2).to(dtype) for k, s in shapes.items()} for _ in range(4)]
    counts = [7, 3, 9, 2]
    opt = S_make(sort)
    ora = O.OracleFedOPT(sort)
    bw = {k: v.to(DEV) for k, v in base0.items()}
    ob = {k: v.clone() for k, v in base0.items()}
    running = 0
    for i, u in enumerate(ups):
        running += counts[i]
        c, oc = S.SortedCache(), S.SortedCache()
        c[f"e{i}"] = S.TR({k: v.to(DEV) for k, v in u.items()}, counts[i])
        oc[f"e{i}"] = S.TR({k: v.clone() for k, v in u.items()}, counts[i])
        before = _counts()
        got = opt.do(bw, c, total=running, num_trainers=4)
        exp = ora.do(ob, oc, total=running)
        torch.cuda.synchronize()
        hits = _diff(before, _counts())
        if i == 1:      # the aliased step: fused, one launch, no generic path
            assert sum(v for k, v in hits.items() if k.startswith("flame_fedopt_reduce_adapt")) == 1, hits
            assert not any(k.startswith("flame_agg_reduce") for k in hits), hits
            S.assert_bitwise(f"eager/{sort}/{dt}/step1/cur", S.to_cpu(got), exp)
        elif i >= 2:
            S.assert_close_fedopt(f"eager/{sort}/{dt}/step{i}/cur", S.to_cpu(got), exp, elementwise=i == 2)
        S.assert_bitwise(f"eager/{sort}/{dt}/step{i}/avg", S.to_cpu(bw), ob)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16, torch.float64, torch.int64,
                                   torch.int32])
def test_device_table_reduction_every_dtype(dtype, monkeypatch):
    """flame_agg_reduce through the device-table launch (engine.ARGMETA off) for every dtype
    the kernel instantiates, 37 clients over a ragged 70,001 + 3-element model, bitwise ==
    the oracle (the kernel-argument launch is test_reduce_vs_oracle_dtypes)."""
    from flame_amd import engine
    O = _oracle()
    monkeypatch.setattr(engine, "ARGMETA", False)
    g = torch.Generator().manual_seed(23)
    n, shapes = 37, {"a": (70_001,), "b": (3,)}
    if dtype.is_floating_point:
        base = {k: torch.randn(s, generator=g, dtype=torch.float64).to(dtype) for k, s in shapes.items()}
        cl = [{k: (torch.randn(s, generator=g, dtype=torch.float64) * 1e-2).to(dtype) for k, s in shapes.items()}
              for _ in range(n)]
    else:
        base = {k: torch.randint(-1000, 1000, s, generator=g, dtype=dtype) for k, s in shapes.items()}
        cl = [{k: torch.randint(-100, 100, s, generator=g, dtype=dtype) for k, s in shapes.items()} for _ in range(n)]
    counts = torch.randint(1, 1000, (n,), generator=g).tolist()
    total = sum(counts)
    exp = {k: v.clone() for k, v in base.items()}
    for k in exp:
        O.reduce_tensor(exp[k], [c[k] for c in cl], [c / total for c in counts])
    cache = S.SortedCache()
    for i in range(n):
        cache[f"{i:03d}"] = S.TR({k: v.to(DEV) for k, v in cl[i].items()}, counts[i])
    before = _counts()
    out = S_make("fedavg").do({k: v.to(DEV) for k, v in base.items()}, cache, total=total)
    torch.cuda.synchronize()
    hits = _diff(before, _counts())
    code = {torch.float32: "f32", torch.bfloat16: "bf16", torch.float16: "f16", torch.float64: "f64",
            torch.int64: "i64", torch.int32: "i32"}[dtype]
    assert hits == {f"flame_agg_reduce/{code}": 1}, hits
    S.assert_bitwise(f"table/{code}", out, exp)


@pytest.mark.parametrize("dt", list(DTS))
@pytest.mark.parametrize("mode", ["fedbuff", "sync"])
def test_hierarchy_lds_groups_kernel_argument_launch(dt, mode):
    """16 middles (>= kHLdsMinMids: LDS-held store groups) small enough for the kernel-argument
    launch -- flame_hier_fedbuff_argmeta/lds -- bitwise == the roles' separate calls on the
    oracle: FedBuff mode (asyncfl middles' FedBuff + scale_add + delta, the top's FedBuff of
    the deltas + scale_add) and sync mode (syncfl middles' FedAvg from their weights, deltas,
    the top's FedAvg of the deltas)."""
    from flame_amd.optimizer.fedbuff import hierarchy_round
    from flame_amd.optimizer.sync_hierarchy import sync_hierarchy_round
    O = _oracle()
    dtype = DTS[dt]
    g = torch.Generator().manual_seed(29)
    M, C, P, rnd = 16, 2, 5_003, 9
    ups = [[(torch.randn(P, generator=g) * 1e-2).to(dtype) for _ in range(C)] for _ in range(M)]
    mid0 = [torch.randn(P, generator=g).to(dtype) for _ in range(M)]
    top0 = torch.randn(P, generator=g).to(dtype)
    counts = [[int(x) for x in torch.randint(1, 100, (C,), generator=g)] for _ in range(M)]
    mids = [{"x": w.to(DEV)} for w in mid0]
    top = {"x": top0.to(DEV)}
    before = _counts()
    if mode == "fedbuff":
        aggs = []
        for m in range(M):
            opt = S_make("fedbuff")
            aggs.append(opt.do_arrivals(None, [S.TR({"x": u.to(DEV)}, 1, rnd - (m + t) % 3)
                                               for t, u in enumerate(ups[m])], version=rnd))
        before = _counts()
        hierarchy_round([(mids[m], aggs[m], C, rnd - m % 2) for m in range(M)], None, version=rnd,
                        top_weights=top, top_goal=M)
    else:
        specs = []
        for m in range(M):
            c = S.SortedCache()
            for t in range(C):
                c[f"{t}"] = S.TR({"x": ups[m][t].to(DEV)}, counts[m][t])
            specs.append((mids[m], c, sum(counts[m])))
        sync_hierarchy_round(specs, top)
    torch.cuda.synchronize()
    hits = _diff(before, _counts())
    assert hits == {f"flame_hier_fedbuff_argmeta/lds/{dt}/{mode}": 1}, hits
    # the oracle: the roles' separate calls
    exp_mids, deltas = [], []
    for m in range(M):
        w = {"x": mid0[m].clone()}
        if mode == "fedbuff":
            fb, agg = O.OracleFedBuff(), None
            for t in range(C):
                c = S.SortedCache()
                c["a"] = S.TR({"x": ups[m][t].clone()}, 1, rnd - (m + t) % 3)
                agg = fb.do(agg, c, total=1, version=rnd)
            deltas.append({"x": O.scale_add_tensor(w["x"], agg["x"], C, want_delta=True)})
        else:
            c = S.SortedCache()
            for t in range(C):
                c[f"{t}"] = S.TR({"x": ups[m][t].clone()}, counts[m][t])
            new = O.OracleFedAvg().do({"x": w["x"].clone()}, c, total=sum(counts[m]))
            deltas.append({"x": new["x"] - w["x"]})
            w = new
        exp_mids.append(w)
    exp_top = {"x": top0.clone()}
    if mode == "fedbuff":
        ot, tagg = O.OracleFedBuff(), None
        for m in range(M):
            c = S.SortedCache()
            c["d"] = S.TR(deltas[m], 1, rnd - m % 2)
            tagg = ot.do(tagg, c, total=1, version=rnd)
        ot.scale_add_agg_weights(exp_top, tagg, M)
    else:
        c = S.SortedCache()
        for m in range(M):
            c[f"mid{m:02d}"] = S.TR(deltas[m], sum(counts[m]))
        O.OracleFedAvg().do(exp_top, c, total=sum(sum(x) for x in counts))
    for m in range(M):
        S.assert_bitwise(f"lds-argmeta/{mode}/{dt}/mid{m}", S.to_cpu(mids[m]), exp_mids[m])
    S.assert_bitwise(f"lds-argmeta/{mode}/{dt}/top", S.to_cpu(top), exp_top)
