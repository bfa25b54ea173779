"""Host-side logic of the drop-in path (no GPU): planning, rates, error behaviour, registry."""
import math

import numpy as np
import pytest
import torch

import scenarios as S
from flame_amd import _native as N
from flame_amd import engine


def test_rate32_matches_torch_scalar_rounding():
    x = torch.ones(1)
    for r in [0.1, 1 / 3, 2000 / 4000, 123 / 517_311, 1 / math.sqrt(3)]:
        assert (x * r).item() == engine.rate32(r)


def test_plan_layout_and_chunks():
    segs = [engine.Seg(1000, out=4096, inp=4096, clients=[8192, 12288]),
            engine.Seg(1, out=8004, inp=8004, clients=[16384, 20480]),
            engine.Seg(0, out=16, inp=16, clients=[32, 48]),
            engine.Seg(5000, out=64, inp=64, clients=[4, 128])]       # client ptr 4: unaligned
    p = engine.plan(N.FLAME_F32, segs, [0.25, 0.75])
    w = p.meta
    assert p.n_segs == 4 and p.n_clients == 2
    chunk = engine.chunk_elems(N.FLAME_F32)
    assert chunk == 1024
    begins = [w[i * 10 + 7] for i in range(4)]
    assert begins == [0, 1, 2, 2]
    assert p.n_chunks == 2 + 5
    flags = [w[i * 10 + 8] for i in range(4)]
    assert flags == [0, N.FLAME_SEG_UNALIGNED, 0, N.FLAME_SEG_UNALIGNED]  # 8004 % 16 != 0
    assert list(w[p.off_clients // 8: p.off_clients // 8 + 8]) == [8192, 12288, 16384, 20480, 32, 48, 4, 128]
    r32 = w[p.off_r32 // 8:p.off_r64 // 8].view(np.float32)
    assert r32[0] == np.float32(0.25) and r32[1] == np.float32(0.75)
    r64 = w[p.off_r64 // 8:].view(np.float64)
    assert list(r64) == [0.25, 0.75]


def test_plan_rejects_ragged_client_rows():
    with pytest.raises(ValueError):
        engine.plan(N.FLAME_F32, [engine.Seg(4, clients=[1]), engine.Seg(4, clients=[1, 2])], [0.5, 0.5])


def test_dtype_support():
    assert engine.dtype_code(torch.bfloat16) == N.FLAME_BF16
    with pytest.raises(TypeError):
        engine.dtype_code(torch.uint8)


def test_fedavg_none_results_need_no_gpu():
    from flame_amd.optimizers import optimizer_provider
    opt = optimizer_provider.get("fedavg")
    base = {"w": torch.ones(3)}
    assert opt.do(base, S.SortedCache(), total=4) is None
    assert opt.agg_weights is base
    c = S.SortedCache()
    c["a"] = S.TR({"w": torch.ones(3)}, 0)
    assert opt.do(base, c, total=0) is None and len(c) == 1
    with pytest.raises(AssertionError):
        opt.do(None, c, total=1)


def test_fedopt_none_returns_current():
    from flame_amd.optimizers import optimizer_provider
    opt = optimizer_provider.get("fedyogi", beta_1=0.5)
    assert opt.beta_1 == 0.5 and opt.beta_2 == 0.99 and opt.eta == 1e-2 and opt.tau == 1e-3
    assert opt.do({"w": torch.ones(2)}, S.SortedCache(), total=3) is None


def test_fedbuff_stale_errors_raise_before_launch():
    from flame_amd.optimizers import optimizer_provider
    opt = optimizer_provider.get("fedbuff")
    c = S.SortedCache()
    c["a"] = S.TR({"w": torch.ones(2)}, 1, 6)
    with pytest.raises(ZeroDivisionError):
        opt.do(None, c, total=1, version=5)
    assert len(c) == 0  # popped before the rate, like the reference
    c["b"] = S.TR({"w": torch.ones(2)}, 1, 9)
    with pytest.raises(ValueError):
        opt.do(None, c, total=1, version=5)
    assert opt.do(None, S.SortedCache(), total=1, version=5) is None


def test_provider_semantics():
    from flame_amd.optimizers import optimizer_provider, ObjectFactory, install, DROP_INS
    with pytest.raises(ValueError):
        optimizer_provider.get("fedsgd")
    f = ObjectFactory()
    install(f)
    ctor = {"fedprox": {"mu": 0.01}, "feddyn": {"alpha": 0.01}, "scaffold": {"k": 3},
            "fedgft": {"fair": "SP", "gamma": 0.5}}
    for k in DROP_INS:
        kw = ctor.get(k, {})
        assert isinstance(f.create(k, **kw), DROP_INS[k])
    assert optimizer_provider.get("fedadam").regularizer.get_term() == 0.0


def test_synth_generator_stats():
    from flame_amd import synth
    x = synth.synth_f32(0, 5, 200_000, 0.01)
    assert abs(float(x.mean())) < 1e-4 and abs(float(x.std()) / 0.01 - 1) < 0.01
    c = synth.counts(1, 256)
    assert c.min() >= 1 and c.max() <= 1000


def test_fedbuff_defers_arrivals_without_launch():
    """do() per arrival only queues (no GPU touched until the aggregate is read)."""
    from flame_amd.optimizers import optimizer_provider
    from flame_amd.optimizer.fedbuff import DeferredAggregate
    opt = optimizer_provider.get("fedbuff")
    agg = None
    for i in range(5):
        c = S.SortedCache()
        c[f"{i}"] = S.TR({"w": torch.ones(3), "b": torch.ones(1)}, 2, 7 - (i % 3))
        agg = opt.do(agg, c, total=2, version=7)
    assert isinstance(agg, DeferredAggregate) and opt.agg_goal_weights is agg
    assert list(agg) == ["w", "b"] and len(agg) == 2 and len(agg._pending) == 5
    with pytest.raises(KeyError):
        c = S.SortedCache()
        c["x"] = S.TR({"zz": torch.ones(1)}, 1, 7)
        opt.do(agg, c, total=1, version=7)
    plain = optimizer_provider.get("fedbuff", defer=False)
    assert plain.defer is False


def test_fedbuff_do_arrivals_matches_per_do_queue():
    """FedBuff.do_arrivals == the role's do() per arrival, before any launch: the same queued
    (weights, rate) pairs in the same order (rates bit-equal to 1 / math.sqrt(...)), the same
    None-start, the same aggregate object when one exists."""
    import math
    from flame_amd.optimizers import optimizer_provider
    from flame_amd.optimizer.fedbuff import DeferredAggregate
    ws = [{"w": torch.full((3,), float(i)), "b": torch.ones(1)} for i in range(9)]
    vers = [17 - (i * 7) % 5 for i in range(9)]
    ref, agg = optimizer_provider.get("fedbuff"), None
    for i in range(9):
        c = S.SortedCache()
        c[f"{i}"] = S.TR(ws[i], 2, vers[i])
        agg = ref.do(agg, c, total=2, version=17)
    opt = optimizer_provider.get("fedbuff")
    got = opt.do_arrivals(None, [S.TR(ws[i], 2, vers[i]) for i in range(9)], version=17)
    assert isinstance(got, DeferredAggregate) and opt.agg_goal_weights is got
    assert [(id(w), r) for w, r in got._pending] == [(id(w), r) for w, r in agg._pending]
    assert [r for _, r in got._pending] == [1 / math.sqrt(1 + 17 - v) for v in vers]
    assert opt.is_agg_weights_none is False and ref.is_agg_weights_none is False
    # onto an existing aggregate: one queue extension, same object
    more = [S.TR(ws[i], 3, 16) for i in range(4)]
    again = opt.do_arrivals(got, more, version=17)
    assert again is got and len(got._pending) == 13
    # a single arrival onto None: a None-start, as one do()
    one = optimizer_provider.get("fedbuff")
    a1 = one.do_arrivals(None, [S.TR(ws[0], 1, 17)], version=17)
    assert one.is_agg_weights_none is True and len(a1._pending) == 1 and a1._pending[0][1] == 1.0
    assert one.do_arrivals(a1, [], version=17) is a1


def test_deferred_aggregate_tracks_one_slab_queue():
    """DeferredAggregate notes when every queued arrival is a whole slot of one slab (pointer
    rows then come from the slot numbers): the slab and the slots in queue order; a plain dict
    or a second slab turns it off; a rejected arrival leaves it as it was; a flush resets it."""
    from flame_amd.optimizers import optimizer_provider

    class FakeSlab:
        def __init__(self):
            self.keys = ["w"]
            self.meta = {"w": (torch.float32, (4,), 4, 0, 1)}

    class Slot(dict):
        __slots__ = ("__weakref__", "slab", "slot", "shapes")

    def slot(slab, i):
        w = Slot(w=torch.empty(0))
        w.slab, w.slot, w.shapes = slab, i, {"w": (4,)}
        return w

    a, b = FakeSlab(), FakeSlab()
    opt = optimizer_provider.get("fedbuff")
    agg = opt.do_arrivals(None, [S.TR(slot(a, i), 1, 3) for i in (5, 2, 9)], version=3)
    assert agg._pend_slab is a and agg._pend_slots == [5, 2, 9]
    with pytest.raises(KeyError):
        bad = Slot(zz=torch.empty(0))
        opt.do_arrivals(agg, [S.TR(slot(a, 1), 1, 3), S.TR({"zz": torch.ones(4)}, 1, 3)], version=3)
    assert agg._pend_slab is a and agg._pend_slots == [5, 2, 9] and len(agg._pending) == 3
    opt.do_arrivals(agg, [S.TR(slot(a, 7), 1, 3)], version=3)
    assert agg._pend_slots == [5, 2, 9, 7]
    opt.do_arrivals(agg, [S.TR(slot(b, 0), 1, 3)], version=3)
    assert agg._pend_slab is False
    agg2 = optimizer_provider.get("fedbuff").do_arrivals(None, [S.TR(slot(a, 0), 1, 3), S.TR({"w": torch.ones(4)}, 1, 3)],
                                                         version=3)
    assert agg2._pend_slab is False
    agg2._clear_pending()
    assert agg2._pend_slab is None and agg2._pend_slots == [] and agg2._pending == []
    del bad


def test_fedbuff_do_arrivals_raises_at_the_stale_arrival():
    """A stale version raises as math does, at its position: earlier arrivals are queued."""
    from flame_amd.optimizers import optimizer_provider
    opt = optimizer_provider.get("fedbuff")
    arr = [S.TR({"w": torch.ones(2)}, 1, 5), S.TR({"w": torch.ones(2)}, 1, 4), S.TR({"w": torch.ones(2)}, 1, 6),
           S.TR({"w": torch.ones(2)}, 1, 1)]
    with pytest.raises(ZeroDivisionError):
        opt.do_arrivals(None, arr, version=5)          # 1 + 5 - 6 == 0 at the third arrival
    assert len(opt.agg_goal_weights._pending) == 2
    arr[2] = S.TR({"w": torch.ones(2)}, 1, 9)
    opt2 = optimizer_provider.get("fedbuff")
    with pytest.raises(ValueError):
        opt2.do_arrivals(None, arr, version=5)         # negative: math domain error
    assert len(opt2.agg_goal_weights._pending) == 2
    with pytest.raises(ValueError):
        optimizer_provider.get("fedbuff").do_arrivals(None, [S.TR({"w": torch.ones(2)}, 0, 5)], version=5)
    opt3 = optimizer_provider.get("fedbuff")
    with pytest.raises(ZeroDivisionError):
        opt3.do_arrivals(None, [S.TR({"w": torch.ones(2)}, 1, 6)], version=5)
    assert opt3.agg_goal_weights is None


def test_fedprox_is_fedavg_with_regularizer():
    from flame_amd.optimizers import optimizer_provider
    from flame_amd.optimizer.fedavg import FedAvg
    opt = optimizer_provider.get("fedprox", mu=0.1)
    assert isinstance(opt, FedAvg) and opt.mu == 0.1
    w = [torch.ones(3), torch.zeros(2)]
    wt = [torch.zeros(3), torch.zeros(2)]
    assert abs(float(opt.regularizer.get_term(w=w, w_t=wt)) - 0.15) < 1e-7


def test_feddyn_save_state_tracks_active_ends():
    """feddyn.py:51-62: history kept for active ends, None for new ones, others dropped."""
    from flame_amd.optimizers import optimizer_provider
    opt = optimizer_provider.get("feddyn", alpha=0.1)
    assert opt.alpha == 0.1 and opt.cld_model is None
    opt.local_param_dict = {"a": {"w": torch.ones(2)}, "b": {"w": torch.zeros(2)}}
    opt.save_state(S._PRE, active_ends=["b", "c"])
    assert list(opt.local_param_dict) == ["b", "c"] and opt.local_param_dict["c"] is None
    opt.save_state(type("S", (), {"value": "post"}), active_ends=[])
    assert list(opt.local_param_dict) == ["b", "c"]
    assert opt.do({"w": torch.zeros(2)}, S.SortedCache(), total=5) is None
    with pytest.raises(AssertionError):
        opt.do(None, S.SortedCache())


def test_scaffold_weight_dict_and_none_paths():
    """scaffold.py:58-79 weight_dict; do() returns None for an empty cache, total 0 or a
    control cache whose length differs -- before consuming anything (:113-119)."""
    from flame_amd.optimizers import optimizer_provider
    opt = optimizer_provider.get("scaffold", k=3)
    opt.save_state(S._PRE, dataset_sizes={"a": 10, "b": 30})
    assert opt.weight_dict == {"a": 0.5, "b": 1.5}
    cache, cc = S.SortedCache(), S.SortedCache()
    cache["a"] = S.TR({"w": torch.ones(2)}, 10)
    assert opt.do({"w": torch.zeros(2)}, cache, total=10, control_cache=cc) is None
    assert opt.do({"w": torch.zeros(2)}, cache, total=0, control_cache=cc) is None
    assert opt.do({"w": torch.zeros(2)}, S.SortedCache(), total=10, control_cache=cc) is None
    assert len(cache) == 1
    with pytest.raises(KeyError):
        opt.do({"w": torch.zeros(2)}, cache, total=10)   # control_cache is required


def test_drop_in_keys_cover_reference_provider():
    """Every key flame's provider registers (optimizers.py:40-48) is a drop-in."""
    from flame_amd.optimizers import DROP_INS
    assert set(DROP_INS) == {"fedavg", "fedadagrad", "fedadam", "fedyogi", "fedbuff", "fedprox",
                             "feddyn", "scaffold", "fedgft"}


def test_plan_per_segment_rates_layout():
    """FLAME_AGG_SEG_RATES: rates32/rates64 are [n_segs][n_clients] row-major."""
    segs = [engine.Seg(10, out=64, inp=64, clients=[128, 256]), engine.Seg(5, out=64, inp=64, clients=[512, 1024])]
    p = engine.plan(0, segs, [[0.5, 0.25], [1 / 3, 0.1]], seg_rates=True)
    assert p.n_clients == 2 and p.n_segs == 2
    r32 = p.meta.view(np.uint8)[p.off_r32:p.off_r32 + 16].view(np.float32)
    assert list(r32) == [np.float32(0.5), np.float32(0.25), np.float32(1 / 3), np.float32(0.1)]
    r64 = p.meta.view(np.uint8)[p.off_r64:p.off_r64 + 32].view(np.float64)
    assert list(r64) == [0.5, 0.25, 1 / 3, 0.1]
    with pytest.raises(ValueError):
        engine.plan(0, segs, [[0.5, 0.25], [0.1]], seg_rates=True)
    with pytest.raises(ValueError):
        engine.plan(0, segs, [[0.5, 0.25]], seg_rates=True)


def test_plan_hier_layout():
    """flame_hier_fedbuff metadata: 8-word segments, [S][M] weight / delta tables,
    [S][M*C] arrival table, fp32 rate rows, goals and top rates at the recorded offsets."""
    M, C = 3, 2
    segs = [engine.HierSeg(3000, mid_w=[16 * (i + 1) for i in range(M)], clients=[4096 * (i + 1) for i in range(M * C)],
                           mid_delta=[0, 32, 48], top_w=64, top_in=0, top_out=80, tile_stride=8192),
            engine.HierSeg(5, mid_w=[96, 112, 8], clients=[1024] * (M * C), top_out=128)]   # mid_w 8: unaligned
    rates = [[0.5, 1 / 3], [1.0, 0.25], [0.7, 0.1]]
    p = engine.plan_hier(N.FLAME_F32, segs, rates, [2, 3, 4], [1.0, 0.5, 1 / 3])
    w = p.meta
    assert (p.n_segs, p.n_mids, p.n_clients) == (2, M, C)
    chunk = engine.chunk_elems(N.FLAME_F32)
    assert p.n_chunks == -(-3000 // chunk) + 1
    assert list(w[0:8]) == [64, 0, 80, 3000, 0, 0, 8192, 0]
    assert list(w[8:16]) == [0, 0, 128, 5, -(-3000 // chunk), N.FLAME_SEG_UNALIGNED, 0, 0]
    o = p.offs
    assert o["mid_w"] == 16 * 8 and o["mid_delta"] == o["mid_w"] + 2 * M * 8
    assert list(w[o["mid_w"] // 8:o["mid_w"] // 8 + M]) == [16, 32, 48]
    assert list(w[o["mid_delta"] // 8:o["mid_delta"] // 8 + 2 * M]) == [0, 32, 48, 0, 0, 0]
    assert list(w[o["clients"] // 8:o["clients"] // 8 + M * C]) == [4096 * (i + 1) for i in range(M * C)]
    f = w.view(np.float32)
    assert list(f[o["mid_rates"] // 4:o["mid_rates"] // 4 + M * C]) == [np.float32(r) for row in rates for r in row]
    assert list(f[o["mid_goal"] // 4:o["mid_goal"] // 4 + M]) == [2.0, 3.0, 4.0]
    assert list(f[o["top_rates"] // 4:o["top_rates"] // 4 + M]) == [np.float32(x) for x in (1.0, 0.5, 1 / 3)]
    with pytest.raises(ValueError):
        engine.plan_hier(N.FLAME_F32, segs, [[0.5, 0.1], [0.2]], [2, 3], [1.0, 1.0])
    with pytest.raises(ValueError):
        engine.plan_hier(N.FLAME_F32, segs, rates, [2, 3], [1.0, 1.0])


class _MC:
    """MetricCollector surface (monitor/metric_collector.py:117-121)."""

    def __init__(self):
        self.state_dict = {}

    def save(self, mtype, alias, value):
        self.state_dict[f"{alias}.{mtype}"] = value


def test_metric_collector_hook_without_launches():
    """An instrumented do() that launches nothing saves nothing and keeps the contract."""
    from flame_amd import metrics
    from flame_amd.optimizers import optimizer_provider
    opt = optimizer_provider.get("fedavg")
    opt.metric_collector = _MC()
    assert opt.do({"w": torch.zeros(3)}, S.SortedCache(), total=0) is None
    metrics.flush()
    assert opt.metric_collector.state_dict == {}
    # every drop-in's entry points are wrapped
    from flame_amd.optimizers import DROP_INS
    for sort, cls in DROP_INS.items():
        assert getattr(cls.do, "__wrapped__", None) is not None, sort


def test_fedgft_bias_matches_reference_fixture(golden):
    """FedGFT.update_bias / get_bias (fedgft.py:50-58, bias.py:74-106) against the values
    the reference produced for the same trainer terms (fedgft_rounds.npz); host arithmetic only."""
    from flame_amd.optimizers import optimizer_provider
    from flame_amd.optimizer.fedavg import FedAvg
    fx = golden("fedgft_rounds.npz")
    m = fx.meta
    for fair in m["fairs"]:
        opt = optimizer_provider.get("fedgft", fair=fair, gamma=m["gamma"])
        assert isinstance(opt, FedAvg) and opt.get_bias() == 0.0
        for r, ends in enumerate(m["rounds"]):
            bm = m["bias"][f"{fair}/r{r}"]
            local = {e: S._LocalBias(*t) for e, t in zip(ends, bm["local"])}
            opt.update_bias(dataset_sizes={e: bm["sizes"][e] for e in ends}, local_biases=local)
            assert S._bias_terms(opt) == bm["global"] and opt.get_bias() == bm["get_bias"]


def test_feddyn_program_merged_and_two_phase():
    """engine.feddyn_program: FedAvg in arrival order, mean in dict order (feddyn.py:96-112)."""
    W, AVG, HIN, HOUT, MEAN = N.FLAME_DYN_W, N.FLAME_DYN_AVG, N.FLAME_DYN_HIN, N.FLAME_DYN_HOUT, N.FLAME_DYN_MEAN
    arr = W | AVG | HOUT
    # arrivals in dict order: one merged list; a None end that does not arrive contributes nothing
    steps, n1 = engine.feddyn_program(["a", "c", "z"], ["a", "b", "c", "d", "z"], {"a", "b"})
    assert steps == [(arr | HIN | MEAN, "a"), (HIN | MEAN, "b"), (arr | MEAN, "c"), (arr | MEAN, "z")]
    assert n1 == len(steps)
    # arrival order differs from dict order: phase 1 = arrivals, phase 2 = the mean in dict order
    steps, n1 = engine.feddyn_program(["a", "c"], ["c", "b", "a"], {"a", "b", "c"})
    assert n1 == 2
    assert steps == [(arr | HIN, "a"), (arr | HIN, "c"), (HIN | MEAN, "c"), (HIN | MEAN, "b"), (HIN | MEAN, "a")]
    meta, n_chunks, offs = engine.plan_feddyn(
        N.FLAME_F32, [engine.DynSeg(5000, out=4096, inp=4096, cld=8192, steps=[(16, 32, 32)] * 5)], [f for f, _ in steps])
    T = engine.chunk_elems(N.FLAME_F32)
    assert n_chunks == -(-5000 // T) and offs["steps"] == 64 and offs["flags"] == 64 + 5 * 3 * 8
    assert list(meta[offs["flags"] // 8:].view(np.uint32)[:5]) == [f for f, _ in steps]


def test_plan_chunk_map_property():
    """Randomised: every non-empty segment owns ceil(numel/chunk) consecutive chunks, the
    chunks tile [0, n_chunks) with no gap or overlap, and the tables sit where the offsets
    say (full and compact blocks) -- the invariants the kernel's chunk -> segment lookup
    and the C ABI's bounds checks rely on."""
    hyp = pytest.importorskip("hypothesis")
    st = hyp.strategies

    @hyp.settings(max_examples=200, deadline=None)
    @hyp.given(numels=st.lists(st.integers(0, 5000), min_size=1, max_size=12),
               n=st.integers(1, 9), code=st.sampled_from([N.FLAME_F32, N.FLAME_BF16, N.FLAME_F16, N.FLAME_F64]),
               compact=st.booleans())
    def check(numels, n, code, compact):
        segs = [engine.Seg(k, out=64 * (i + 1), inp=64 * (i + 1), clients=[4096 * (i * n + j + 1) for j in range(n)])
                for i, k in enumerate(numels)]
        rates = [1.0 / (j + 2) for j in range(n)]
        p = engine.plan(code, segs, rates, compact=compact)
        w = p.meta
        chunk = engine.chunk_elems(code)
        nxt = 0
        for i, k in enumerate(numels):
            assert w[i * N.SEGMENT_INT64S + 6] == k
            assert w[i * N.SEGMENT_INT64S + 7] == nxt
            nxt += -(-k // chunk)
        assert p.n_chunks == max(nxt, 1)
        tab = w[p.off_clients // 8:p.off_clients // 8 + len(segs) * n]
        assert list(tab) == [c for s in segs for c in s.clients]
        if compact:
            assert (p.off_r32 == -1) == (code == N.FLAME_F64) and (p.off_r64 == -1) == (code != N.FLAME_F64)
        off = p.off_r64 if p.off_r32 < 0 else p.off_r32
        dt = np.float64 if p.off_r32 < 0 else np.float32
        got = w.view(np.uint8)[off:off + n * np.dtype(dt).itemsize].view(dt)
        assert list(got) == [dt(r) for r in rates]
        assert off + n * np.dtype(dt).itemsize <= w.nbytes

    check()


def test_plan_hier_property():
    """Randomised flame_hier_fedbuff metadata: the seven tables follow one another with no
    gap, each at its recorded offset and of its [S][M] / [S][M*C] / [M*C] / [M] size, and
    the chunks tile [0, n_chunks) segment by segment."""
    hyp = pytest.importorskip("hypothesis")
    st = hyp.strategies

    @hyp.settings(max_examples=150, deadline=None)
    @hyp.given(numels=st.lists(st.integers(0, 9000), min_size=1, max_size=6), M=st.integers(1, 5),
               C=st.integers(1, 6), delta=st.booleans(), code=st.sampled_from([N.FLAME_F32, N.FLAME_BF16, N.FLAME_F16]))
    def check(numels, M, C, delta, code):
        segs = [engine.HierSeg(k, mid_w=[256 * (i * M + m + 1) for m in range(M)],
                               clients=[1 << 20 | 256 * (i * M * C + j) for j in range(M * C)],
                               mid_delta=[1 << 24 | 256 * (i * M + m) for m in range(M)] if delta else None,
                               top_out=1 << 28 | 256 * i)
                for i, k in enumerate(numels)]
        rates = [[1.0 / (m + c + 2) for c in range(C)] for m in range(M)]
        goals = list(range(2, M + 2))
        tops = [1.0 / (m + 1) for m in range(M)]
        p = engine.plan_hier(code, segs, rates, goals, tops)
        S, o, w = len(segs), p.offs, p.meta
        sizes = {"segs": S * engine.HSEG_WORDS * 8, "mid_w": S * M * 8, "mid_delta": S * M * 8,
                 "clients": S * M * C * 8, "mid_rates": -(-M * C // 2) * 8, "mid_goal": -(-M // 2) * 8,
                 "top_rates": -(-M // 2) * 8}
        at = 0
        for nm in ["segs", "mid_w", "mid_delta", "clients", "mid_rates", "mid_goal", "top_rates"]:
            assert o[nm] == at, nm
            at += sizes[nm]
        assert at == w.nbytes
        assert list(w[o["clients"] // 8:o["clients"] // 8 + S * M * C]) == [c for s in segs for c in s.clients]
        dt = list(w[o["mid_delta"] // 8:o["mid_delta"] // 8 + S * M])
        assert dt == ([d for s in segs for d in s.mid_delta] if delta else [0] * (S * M))
        f = w.view(np.float32)
        assert list(f[o["mid_goal"] // 4:o["mid_goal"] // 4 + M]) == [float(g) for g in goals]
        chunk, nxt = engine.chunk_elems(code), 0
        for i, k in enumerate(numels):
            assert w[i * engine.HSEG_WORDS + 3] == k and w[i * engine.HSEG_WORDS + 4] == nxt
            nxt += -(-k // chunk)
        assert p.n_chunks == max(nxt, 1) and (p.n_mids, p.n_clients, p.n_segs) == (M, C, S)

    check()


def test_compact_block_size_prediction():
    """engine._launch_reduce decides kernel-argument vs uploaded metadata from the compact
    block's size before building it; the prediction must equal the built size."""
    import itertools
    for code, S_, n, seg_rates in itertools.product([N.FLAME_F32, N.FLAME_BF16, N.FLAME_F64, N.FLAME_I64],
                                                    [1, 2, 5], [0, 1, 2, 3, 255, 256], [False, True]):
        segs = [engine.Seg(100, out=64, inp=64, clients=[4096] * n) for _ in range(S_)]
        rates = [[0.5] * n for _ in range(S_)] if seg_rates else [0.5] * n
        p = engine.plan(code, segs, rates, seg_rates=seg_rates, compact=True)
        assert p.meta.nbytes == engine.compact_meta_bytes(code, S_, n, seg_rates), (code, S_, n, seg_rates)


# ------------------------------------------------------------------ eager FedAvg deferral
def test_eager_fedavg_defer_queues_one_launch(golden, monkeypatch):
    """FedAvg(defer=True) under the eager caller (eager_syncfl/top_aggregator.py:36-90): the
    arrivals queue with their own count/total and reach the engine as ONE accumulate call on
    the first read; the oracle as that call's arithmetic reproduces the reference fixture's
    final state bitwise.  An empty do() flushes first (None, base already written)."""
    from oracle import oracle as O
    import scenarios as S
    from flame_amd.optimizer import fedavg as F

    calls = []

    def accumulate(base, entries, key_groups=None, after_group=None):
        calls.append(len(entries))
        for k in base:
            O.reduce_tensor(base[k], [w[k] for w, _ in entries], [r for _, r in entries])

    monkeypatch.setattr(F.engine, "accumulate", accumulate)
    fx = golden("fedavg_eager.npz")
    m = fx.meta
    opt = F.FedAvg(defer=True)
    base = {k: v.clone() for k, v in fx.weights("base").items()}
    cache = S.SortedCache()
    total, out = 0, None
    for step, (e, c) in enumerate(zip(m["end_ids"], m["counts"])):
        total += c
        cache[e] = S.TR(fx.weights(f"client{step}"), c)
        out = opt.do(base, cache, total=total, num_trainers=m["n"])
        assert isinstance(out, F.DeferredWeights) and out.pending == step + 1
    assert calls == []
    last = len(m["end_ids"]) - 1
    S.assert_bitwise("final", dict(out.items()), fx.weights(f"after{last}"))
    assert calls == [len(m["end_ids"])]
    assert opt.do(base, S.SortedCache(), total=total) is None and out.pending == 0
    # the non-deferred default keeps the reference's return (the base dict itself)
    cache["z"] = S.TR(fx.weights("client0"), 1)
    assert F.FedAvg().do(base, cache, total=1) is base and calls[-1] == 1


def test_eager_fedavg_defer_raises_at_the_bad_arrival(monkeypatch):
    """A queued arrival with an unknown key or an illegal in-place promotion raises from the
    do() that brings it, as the reference's per-arrival add would (fedavg.py:93-104)."""
    import pytest
    import scenarios as S
    from flame_amd.optimizer import fedavg as F
    monkeypatch.setattr(F.engine, "accumulate", lambda *a, **k: None)
    opt = F.FedAvg(defer=True)
    base = {"w": torch.zeros(4, dtype=torch.bfloat16), "n": torch.tensor(1)}
    c = S.SortedCache()
    c["a"] = S.TR({"w": torch.ones(4, dtype=torch.bfloat16), "n": torch.tensor(2)}, 1)
    out = opt.do(base, c, total=1)
    c["b"] = S.TR({"w": torch.ones(4), "n": torch.tensor(1.5)}, 1)   # int64 += f32: raises
    with pytest.raises(RuntimeError, match="can't be cast"):
        opt.do(base, c, total=2)
    c = S.SortedCache()
    c["c"] = S.TR({"zz": torch.ones(4)}, 1)
    with pytest.raises(KeyError):
        opt.do(base, c, total=3)
    assert out.pending == 1


def test_deferred_queues_free_their_arrivals_without_the_cyclic_gc(monkeypatch):
    """A deferred aggregate holds its optimizer weakly: dropping the optimizer and the
    aggregate frees the queued arrivals at once (slab slots return to the slab), with the
    cyclic garbage collector off."""
    import gc
    import weakref
    import scenarios as S
    from flame_amd.optimizer import fedavg as F, fedbuff as B

    class W(dict):
        pass
    monkeypatch.setattr(F.engine, "accumulate", lambda *a, **k: None)
    gc.disable()
    try:
        w = W(x=torch.ones(3))
        ref = weakref.ref(w)
        fb = B.FedBuff()
        c = S.SortedCache()
        c["a"] = S.TR(w, 1, 0)
        agg = fb.do(None, c, total=1, version=0)
        assert agg._pending
        del w, c, fb, agg
        assert ref() is None, "FedBuff's queue outlived its optimizer and aggregate"
        w = W(x=torch.ones(3))
        ref = weakref.ref(w)
        fa = F.FedAvg(defer=True)
        c = S.SortedCache()
        c["a"] = S.TR(w, 1)
        out = fa.do({"x": torch.zeros(3)}, c, total=1)
        assert out.pending == 1
        del w, c, fa, out
        assert ref() is None, "FedAvg's queue outlived its optimizer"
    finally:
        gc.enable()


def test_deferred_aggregates_pickle_as_plain_dicts(monkeypatch):
    """torch.save / pickle of a deferred result (eager FedAvg, FedBuff) reduces the queue
    and stores an OrderedDict of tensors, loadable with weights_only=True (the optimizer is
    held weakly and is not pickled)."""
    import io
    import scenarios as S
    from flame_amd.optimizer import fedavg as F, fedbuff as B
    from oracle import oracle as O

    def accumulate(base, entries, key_groups=None, after_group=None, device=None):
        for k in base:
            O.reduce_tensor(base[k], [w[k] for w, _ in entries], [r for _, r in entries])
    monkeypatch.setattr(F.engine, "accumulate", accumulate)
    opt = F.FedAvg(defer=True)
    c = S.SortedCache()
    c["a"] = S.TR({"x": torch.ones(4)}, 1)
    out = opt.do({"x": torch.zeros(4)}, c, total=2)
    buf = io.BytesIO()
    torch.save(out, buf)
    back = torch.load(io.BytesIO(buf.getvalue()), weights_only=True)
    assert isinstance(back, dict) and torch.equal(back["x"], torch.full((4,), 0.5))
    fb = B.FedBuff()
    monkeypatch.setattr(B.engine, "first_tmp", lambda w, r, **k: {kk: v * r for kk, v in w.items()})
    c = S.SortedCache()
    c["a"] = S.TR({"x": torch.ones(4)}, 1, 0)
    agg = fb.do(None, c, total=1, version=0)
    monkeypatch.setattr(B.engine, "pick_device", lambda *a, **k: torch.device("cpu"))
    monkeypatch.setattr(B.engine, "reduce_", lambda outs, bases, clients, rates, **k: [
        o.copy_(cl[0] * rates[0]) for o, cl in zip(outs, clients)])
    buf = io.BytesIO()
    torch.save(agg, buf)
    back = torch.load(io.BytesIO(buf.getvalue()), weights_only=True)
    assert isinstance(back, dict) and torch.equal(back["x"], torch.ones(4))


def test_shard_collective_failure_names_rank_and_wave():
    """A failing all-gather (or its wait) re-raises naming this rank and the wave, so an N>1
    bench that dies in a collective says where (bench.py exits non-zero with it)."""
    import pytest
    from flame_amd import shard
    comm = shard._Comm()
    comm.dist, comm.rank, comm.world, comm.backend = object(), 3, 8, "nccl"

    def boom(pairs, wave):
        raise RuntimeError("NCCL error: unhandled system error")
    comm._all_gather_inplace = boom
    with pytest.raises(RuntimeError, match=r"rank 3 of 8 \(nccl\): all-gather of wave 2 failed"):
        comm.all_gather_inplace([(None, None)], wave=2)

    class W:
        def wait(self):
            raise RuntimeError("timeout")
    comm._works = [(1, W())]
    with pytest.raises(RuntimeError, match=r"rank 3 of 8 \(nccl\): wait on the all-gather of wave 1 failed"):
        comm.wait()


def test_plan_carries_caller_segment_flags():
    """A segment's caller flags (FLAME_SEG_CUR_IS_AVG: the eager caller's aliased FedOPT step)
    land in the flags word next to the computed FLAME_SEG_UNALIGNED bit."""
    from flame_amd import engine
    from flame_amd import _native as N
    segs = [engine.Seg(4096, out=4096, inp=4096, cur=0, cur_out=8192, m=12288, v=16384, clients=[20480],
                       flags=N.FLAME_SEG_CUR_IS_AVG),
            engine.Seg(4096, out=4096, inp=4096, cur=4100, cur_out=8192, m=12288, v=16384, clients=[20480])]
    p = engine.plan(N.FLAME_F32, segs, [1.0])
    head = p.meta[:2 * engine.SEG_WORDS].reshape(2, engine.SEG_WORDS)
    assert int(head[0, 8]) == N.FLAME_SEG_CUR_IS_AVG                 # aligned, aliased
    assert int(head[1, 8]) == N.FLAME_SEG_UNALIGNED                  # cur at 4100: not 16-byte aligned


def _fake_chain_kernels(monkeypatch):
    """CPU stand-ins for the FedAvg reduction and flame_fedopt_chain, written with the oracle's
    C restatement, so FedOPT(defer=True)'s queue logic runs without a GPU."""
    from oracle import oracle as O
    from flame_amd.optimizer import fedopt as FO

    def accumulate(base, entries, **kw):
        for k in base:
            ws = [(w[k], r) for w, r in entries if k in w]
            O.reduce_tensor(base[k], [w for w, _ in ws], [r for _, r in ws])
        for gi in range(len(kw.get("key_groups") or ())):
            kw["after_group"](gi)

    launches = []

    def chain(variant, base, cur, cur_out, m, v, clients, rates, step_end, hyper, state_zero, first_aliased):
        launches.append((len(rates), sum(step_end)))
        for s in range(len(base)):
            b, alias = base[s], first_aliased[s]
            c = None if alias else cur[s].clone()
            if state_zero:
                m[s].zero_()
                v[s].zero_()
            for i, r in enumerate(rates):
                O.reduce_tensor(b, [clients[s][i]], [r])
                if step_end[i]:
                    c = O.adapt_tensor(variant, b, b.clone() if alias else c, m[s], v[s], hyper)
                    alias = False
            cur_out[s].copy_(b if alias else c)

    monkeypatch.setattr(FO.engine, "accumulate", accumulate)
    monkeypatch.setattr(FO.engine, "fedopt_chain_", chain)
    monkeypatch.setattr(FO, "_chain_tensors", lambda w: all(t.dtype == torch.float32 for t in w.values()))
    return launches


@pytest.mark.parametrize("sort", ["fedadam", "fedyogi", "fedadagrad"])
def test_fedopt_defer_queue_logic(monkeypatch, sort):
    """FedOPT(defer=True)'s host side against the oracle's per-call sequence, bitwise, with the
    kernels swapped for CPU stand-ins (the GPU tests check the kernels): the passthrough runs at
    once, the round's calls queue and run at the first read, a new base lands the queue, a result
    held across later calls keeps ITS values (the queue is cut there), m_t / v_t reads run it."""
    from oracle import oracle as O
    from flame_amd.optimizer.fedopt import DeferredCurrent
    from flame_amd.optimizers import optimizer_provider
    launches = _fake_chain_kernels(monkeypatch)
    g = torch.Generator().manual_seed(3)
    w0 = {"a": torch.randn(37, generator=g), "b": torch.randn(5, generator=g)}
    ups = [[({k: torch.randn(v.shape, generator=g) * 1e-2 for k, v in w0.items()}, 1 + 7 * i) for i in range(5)]
           for _ in range(2)]
    amd, ora = optimizer_provider.get(sort, defer=True), O.OracleFedOPT(sort)
    wa, wo = {k: v.clone() for k, v in w0.items()}, {k: v.clone() for k, v in w0.items()}
    held_a, held_o = [], []
    for r, calls in enumerate(ups):
        ba, bo = {k: v.clone() for k, v in dict(wa).items()}, {k: v.clone() for k, v in dict(wo).items()}
        total = 0
        for i, (w, c) in enumerate(calls):
            total += c
            ca, co = S.SortedCache(), S.SortedCache()
            ca[f"e{i}"] = S.TR({k: v.clone() for k, v in w.items()}, c)
            co[f"e{i}"] = S.TR({k: v.clone() for k, v in w.items()}, c)
            oa, oo = amd.do(ba, ca, total=total), ora.do(bo, co, total=total)
            assert len(ca) == 0, "a queued call pops its cache as the reference does"
            if r == 0 and i == 0:
                assert oa is ba and not launches          # the passthrough: the base itself, at once
            else:
                assert isinstance(oa, DeferredCurrent)
            if i == 2:
                held_a.append(oa)
                held_o.append({k: v.clone() for k, v in oo.items()})
        n_before = len(launches)
        S.assert_bitwise(f"{sort}/r{r}/current", {k: oa[k] for k in oa}, oo)   # the read runs the queue
        S.assert_bitwise(f"{sort}/r{r}/base", ba, bo)
        S.assert_bitwise(f"{sort}/r{r}/m", amd.m_t, ora.m_t)
        S.assert_bitwise(f"{sort}/r{r}/v", amd.v_t, ora.v_t)
        # one stand-in launch per stretch: cut after the held call (i = 2) and at the end
        assert [n for n, _ in launches[n_before:]] == ([2, 2] if r == 0 else [3, 2]), launches
        wa, wo = oa, oo
    for j, (h, ref) in enumerate(zip(held_a, held_o)):
        S.assert_bitwise(f"{sort}/held{j}", {k: h[k] for k in h}, ref)


def test_fedopt_defer_replays_ineligible_calls(monkeypatch):
    """A call the chain cannot take (a key subset) lands the queue and goes through the per-call
    path with the entries it popped: the per-call path sees them in the same order."""
    from flame_amd.optimizer import fedopt as FO
    from flame_amd.optimizers import optimizer_provider
    _fake_chain_kernels(monkeypatch)
    seen = []
    monkeypatch.setattr(FO.FedOPT, "_do_fused",
                        lambda self, base, cache, total, *a: seen.append(list(cache.iterkeys())) or {"x": 1})
    opt = optimizer_provider.get("fedadam", defer=True)
    base = {"a": torch.zeros(4), "b": torch.zeros(2)}
    c = S.SortedCache()
    c["x0"] = S.TR({"a": torch.ones(4), "b": torch.ones(2)}, 1)
    assert opt.do(base, c, total=1) is base                      # passthrough
    c["x1"] = S.TR({"a": torch.ones(4), "b": torch.ones(2)}, 1)
    out = opt.do(base, c, total=2)
    assert opt._chain is not None and opt._chain.n_entries == 1
    c["x2"] = S.TR({"a": torch.ones(4)}, 1)                      # a key subset: not for the chain
    c["x3"] = S.TR({"a": torch.ones(4)}, 2)
    assert opt.do(base, c, total=5) == {"x": 1}
    assert opt._chain is None and seen == [["x2", "x3"]] and out._value is not None
