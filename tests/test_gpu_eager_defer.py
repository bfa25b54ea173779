"""GPU: eager FedAvg batched into one launch (``FedAvg(defer=True)``).

The eager top aggregator (eager_syncfl/top_aggregator.py:36-90) calls ``do()`` once per
arrival on the same ``base_weights`` with the running total; the deferred drop-in queues
the arrivals (each with its own ``count / total``) and reduces them in one launch when the
result is first read.  Checked bitwise against the reference-generated
``fedavg_eager.npz`` and against the per-arrival drop-in (``defer=False``).
"""
import copy
import gc

import pytest
import torch

import scenarios as S

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _native_loaded():
    from flame_amd import _native
    _native.lib()
    assert torch.cuda.is_available()


def _fedavg(**kw):
    from flame_amd.optimizers import optimizer_provider
    return optimizer_provider.get("fedavg", **kw)


@pytest.mark.oracle
def test_eager_deferred_golden_one_launch(golden):
    """Every arrival queued (base untouched until the read), the final model == the
    reference's state after the last arrival, bitwise."""
    from flame_amd.optimizer.fedavg import DeferredWeights
    fx = golden("fedavg_eager.npz")
    m = fx.meta
    opt = _fedavg(defer=True)
    base = S.to_dev(fx.weights("base"), DEV)
    before = S.to_cpu(base)
    cache = S.SortedCache()
    total = 0
    out = None
    for step, (e, c) in enumerate(zip(m["end_ids"], m["counts"])):
        total += c
        cache[e] = S.TR(S.to_dev(fx.weights(f"client{step}"), DEV), c)
        out = opt.do(base, cache, total=total, num_trainers=m["n"])
        assert isinstance(out, DeferredWeights) and out.pending == step + 1
        assert len(cache) == 0
    S.assert_bitwise("queued: base not yet written", S.to_cpu(base), before)
    last = len(m["end_ids"]) - 1
    got = {k: out[k] for k in out}           # the read reduces the queue (one launch per dtype)
    assert out.pending == 0 and out.materialize() is base
    S.assert_bitwise("final", got, fx.weights(f"after{last}"))
    S.assert_bitwise("base in place", base, fx.weights(f"after{last}"))


def _model(g):
    from flame_amd import engine
    T = engine.chunk_elems(0)
    return {"big": torch.randn(3 * T + 17, generator=g), "bf": torch.randn(2 * 2048 + 3, generator=g).bfloat16(),
            "h": torch.randn(4099, generator=g).half(), "mat": torch.randn(33, 65, generator=g),
            "tiny": torch.randn(5, generator=g), "nbt": torch.tensor(7, dtype=torch.int64)}


def _update(g, tmpl, i):
    return {k: (torch.randn(v.shape, generator=g) * 1e-2).to(v.dtype) if v.is_floating_point()
            else torch.tensor(3 * i + 1, dtype=v.dtype) for k, v in tmpl.items()}


@pytest.mark.parametrize("placement", ["slab", "hbm", "tensors"])
def test_eager_deferred_equals_per_arrival(placement):
    """Mixed dtypes (f32 / bf16 / f16 / int64), a device cache or plain tensors, the eager
    running total, a queue bound that flushes mid-round, an empty do() (None: the queue
    lands first), a read in the middle and a deepcopy of the result for the next round:
    deferred == one launch per arrival, bitwise, round after round."""
    from flame_amd.ingest import DeviceUpdateCache
    g = torch.Generator().manual_seed(21)
    tmpl = _model(g)
    a, b = _fedavg(defer=True, max_pending=7), _fedavg(defer=False)
    wa = {k: v.to(DEV) for k, v in tmpl.items()}
    wb = {k: v.to(DEV) for k, v in tmpl.items()}
    for rnd in range(2):
        ba, bb = copy.deepcopy(wa), copy.deepcopy(wb)       # eager: base = deepcopy(self.weights)
        ca = DeviceUpdateCache(device=DEV, placement=placement, capacity=32) if placement != "tensors" \
            else S.SortedCache()
        cb = S.SortedCache()
        total = 0
        n = 19
        ra = rb = None
        for i in range(n):
            c = 5 + (7 * i) % 11
            total += c
            up = _update(g, tmpl, i)
            ca[f"e{i:02d}"] = S.TR({k: v.to(DEV) for k, v in up.items()}, c)
            cb[f"e{i:02d}"] = S.TR({k: v.to(DEV) for k, v in up.items()}, c)
            ra = a.do(ba, ca, total=total, num_trainers=n)
            rb = b.do(bb, cb, total=total, num_trainers=n)
            assert rb is bb
            if rnd == 0 and i == 9:
                # an empty round-trip: the reference returns None and has already written base
                assert a.do(ba, S.SortedCache(), total=total) is None
                assert b.do(bb, S.SortedCache(), total=total) is None
                S.assert_bitwise(f"r{rnd} after None", S.to_cpu(ba), S.to_cpu(bb))
            if rnd == 1 and i == 12:
                S.assert_bitwise(f"r{rnd} mid read", {"big": ra["big"]}, {"big": bb["big"].cpu()})
        wa = copy.deepcopy(ra)        # the role keeps the returned object; deepcopy flushes
        wb = rb
        assert type(wa) is dict
        S.assert_bitwise(f"r{rnd}", S.to_cpu(wa), S.to_cpu(wb))
    if placement == "slab":
        del ra, ba, ca
        gc.collect()


def test_eager_deferred_new_base_flushes_old():
    """A do() with another base dict reduces the queue into the old one first; a
    DeferredWeights handed back as base_weights is materialised."""
    g = torch.Generator().manual_seed(5)
    tmpl = {"w": torch.randn(10_000, generator=g)}
    a, b = _fedavg(defer=True), _fedavg()
    b1a, b1b = {"w": tmpl["w"].to(DEV)}, {"w": tmpl["w"].to(DEV)}
    ups = [{"w": (torch.randn(10_000, generator=g) * 1e-2).to(DEV)} for _ in range(4)]
    for i in range(2):
        ca, cb = S.SortedCache(), S.SortedCache()
        ca["x"], cb["x"] = S.TR(ups[i], 2 + i), S.TR(ups[i], 2 + i)
        r1 = a.do(b1a, ca, total=5)
        b.do(b1b, cb, total=5)
    b2a, b2b = {"w": tmpl["w"].to(DEV) * 2}, {"w": tmpl["w"].to(DEV) * 2}
    ca, cb = S.SortedCache(), S.SortedCache()
    ca["y"], cb["y"] = S.TR(ups[2], 3), S.TR(ups[2], 3)
    r2 = a.do(b2a, ca, total=3)
    b.do(b2b, cb, total=3)
    assert r1.pending == 0, "the first base's queue lands when another base arrives"
    S.assert_bitwise("old base", S.to_cpu(b1a), S.to_cpu(b1b))
    ca, cb = S.SortedCache(), S.SortedCache()
    ca["z"], cb["z"] = S.TR(ups[3], 1), S.TR(ups[3], 1)
    r3 = a.do(r2, ca, total=4)          # the returned Mapping passed back as base
    b.do(b2b, cb, total=4)
    assert r3.materialize() is b2a
    S.assert_bitwise("new base", S.to_cpu(dict(r3.items())), S.to_cpu(b2b))


def test_deferred_flush_reports_to_metric_collector():
    """The launch a deferred eager FedAvg (and a deferred FedBuff aggregate) makes when it is
    read, outside any do(), still reaches the optimizer's metric_collector."""
    from flame_amd import metrics

    class MC:
        def __init__(self):
            self.state_dict = {}

        def save(self, mtype, alias, value):
            self.state_dict[f"{alias}.{mtype}"] = value

    g = torch.Generator().manual_seed(9)
    opt = _fedavg(defer=True)
    opt.metric_collector = MC()
    base = {"x": torch.randn(50_001, generator=g).to(DEV)}
    total, out = 0, None
    for i in range(5):
        total += 3 + i
        c = S.SortedCache()
        c[f"e{i}"] = S.TR({"x": (torch.randn(50_001, generator=g) * 1e-2).to(DEV)}, 3 + i)
        out = opt.do(base, c, total=total)
    assert out.pending == 5
    _ = out["x"]
    metrics.flush()
    sd = opt.metric_collector.state_dict
    assert sd["fedavg.flame_agg_reduce.launches"] == 1, sd
    from flame_amd.optimizers import optimizer_provider
    fb = optimizer_provider.get("fedbuff")
    fb.metric_collector = MC()
    agg = None
    for i in range(4):
        c = S.SortedCache()
        c["t"] = S.TR({"x": (torch.randn(50_001, generator=g) * 1e-2).to(DEV)}, 1, 7)
        agg = fb.do(agg, c, total=1, version=7)
    _ = agg["x"]
    metrics.flush()
    assert fb.metric_collector.state_dict.get("fedbuff.flame_agg_reduce.launches") == 1, fb.metric_collector.state_dict
