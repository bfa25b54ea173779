"""FedOPT(defer=True)'s queue bookkeeping on the host (no GPU: the chain launch is replaced).

* A failed chain launch leaves the optimizer's state where it was (m_t / v_t not replaced by
  unwritten buffers) and every queued result re-raises the failure when read.
* An eager arrival with nothing to aggregate (empty cache, or total 0) returns the queued
  chain's last result without cutting the chain: one launch per round; the
  reference returns current_weights unchanged there (fedopt.py:80-85, fedavg.py:72-73).
"""
import pytest
import torch

from flame_amd import engine
from flame_amd.optimizer import fedopt as F
from flame_amd.optimizers import optimizer_provider


class TR:
    def __init__(self, weights, count):
        self.weights, self.count, self.version = weights, count, 0


class Cache(dict):
    def iterkeys(self):
        return iter(sorted(self))


@pytest.fixture
def host_chain(monkeypatch):
    """The deferred path over CPU tensors: the queue's eligibility check accepts them and the
    chain launch is a recorder that fills its outputs like the kernel would (or raises)."""
    monkeypatch.setattr(F, "_chain_tensors", lambda w: True)
    calls = []

    def fake_chain(variant, base, cur, cur_out, m, v, clients, rates, step_end, hyper, state_zero, first_aliased):
        calls.append(len(rates))
        if getattr(fake_chain, "fail", None):
            raise RuntimeError(fake_chain.fail)
        for b, o, mm, vv in zip(base, cur_out, m, v):
            o.copy_(b + 1)
            mm.fill_(0.5)
            vv.fill_(0.25)
    monkeypatch.setattr(engine, "fedopt_chain_", fake_chain)
    return fake_chain, calls


def _after_passthrough(sort="fedadam"):
    opt = optimizer_provider.get(sort, defer=True)
    base = {"w": torch.zeros(8)}
    opt._current = base                 # the state right after round 1's passthrough (current IS base)
    return opt, base


def _arrive(opt, base, i, count):
    c = Cache()
    c[f"e{i}"] = TR({"w": torch.full((8,), float(i))}, count)
    return opt.do(base, c, total=10)


def test_failed_chain_keeps_state_and_results_reraise(host_chain):
    fake, calls = host_chain
    fake.fail = "launch refused"
    opt, base = _after_passthrough()
    r1 = _arrive(opt, base, 1, 3)
    r2 = _arrive(opt, base, 2, 4)
    assert isinstance(r1, F.DeferredCurrent) and isinstance(r2, F.DeferredCurrent) and calls == []
    with pytest.raises(RuntimeError, match="launch refused"):
        r2["w"]                                      # the read runs the queue: the launch fails
    assert opt._m is None and opt._v is None       # no unwritten m / v adopted as state
    assert opt.m_t is None and opt.v_t is None
    assert opt.current_weights is base             # still the passthrough's state
    for r in (r1, r2):
        with pytest.raises(RuntimeError, match="did not run: RuntimeError: launch refused"):
            r.materialize()


def test_failure_after_a_cut_keeps_the_cut(host_chain):
    """A held result cuts the queue; when the second stretch's launch fails, the state is the
    first stretch's and only the later result re-raises."""
    fake, calls = host_chain
    opt, base = _after_passthrough("fedyogi")
    r1 = _arrive(opt, base, 1, 3)
    r2 = _arrive(opt, base, 2, 4)
    orig = engine.fedopt_chain_

    def second_fails(*a, **k):
        if calls:
            calls.append("x")
            raise RuntimeError("second stretch")
        return orig(*a, **k)
    engine.fedopt_chain_ = second_fails
    try:
        with pytest.raises(RuntimeError, match="second stretch"):
            r2["w"]
    finally:
        engine.fedopt_chain_ = orig
    assert torch.equal(r1["w"], torch.ones(8))     # the first stretch ran: its result stands
    assert opt._current is r1.materialize()
    assert torch.equal(opt._m["w"], torch.full((8,), 0.5))
    with pytest.raises(RuntimeError, match="did not run"):
        r2.materialize()


@pytest.mark.parametrize("hold", [False, True])
@pytest.mark.parametrize("empty", ["cache", "total"])
def test_nothing_to_aggregate_does_not_cut_the_chain(host_chain, empty, hold):
    fake, calls = host_chain
    opt, base = _after_passthrough("fedadagrad")
    results = [_arrive(opt, base, 1, 3)]
    c = Cache()
    if empty == "total":
        c["z"] = TR({"w": torch.ones(8)}, 0)
    results.append(opt.do(base, c, total=0 if empty == "total" else 10))
    assert len(c) == (1 if empty == "total" else 0)     # total 0: nothing popped (fedavg.py:72-73)
    results.append(_arrive(opt, base, 2, 4))
    assert isinstance(results[1], F.DeferredCurrent) and calls == []
    last = results.pop()
    held = results if hold else []
    del results
    final = dict(last)
    if hold:       # held results cut the queue at their call (both name the first call)
        assert calls == [1, 1], calls
        assert held[1]["w"] is held[0]["w"]             # == current_weights after the first call
    else:          # one launch for the round: the empty arrival did not cut it
        assert calls == [2], calls
    assert opt.current_weights["w"] is final["w"]


@pytest.mark.parametrize("trailing", [False, True])
def test_agg_weights_after_an_empty_arrival(host_chain, trailing):
    """the reference's do() sets agg_weights = FedAvg.do(...) = None for an arrival with
    nothing to aggregate (fedopt.py:80-85); the deferred path matches once the queue has run -- and
    a later real arrival makes agg_weights the base again."""
    fake, calls = host_chain
    opt, base = _after_passthrough("fedadam")
    _arrive(opt, base, 1, 3)
    last = opt.do(base, Cache(), total=10)            # empty arrival, queued chain not cut
    if trailing:
        last = _arrive(opt, base, 2, 4)
    dict(last)
    assert calls == [2 if trailing else 1]
    if trailing:
        assert opt.agg_weights is base
    else:
        assert opt.agg_weights is None
        assert opt.current_weights is not None       # do() returned current_weights, as the reference


def test_partial_launch_failure_poisons_the_optimizer(host_chain):
    """when a later dtype group's launch fails after an earlier one ran (engine marks the
    exception flame_partial), m / v / base disagree across keys: every later call refuses."""
    fake, calls = host_chain
    opt, base = _after_passthrough("fedyogi")
    r = _arrive(opt, base, 1, 3)
    orig = engine.fedopt_chain_

    def partial(*a, **k):
        e = RuntimeError("bf16 group refused")
        e.flame_partial = True
        raise e
    engine.fedopt_chain_ = partial
    try:
        with pytest.raises(RuntimeError, match="bf16 group refused"):
            r["w"]
    finally:
        engine.fedopt_chain_ = orig
    with pytest.raises(RuntimeError, match="re-create the optimizer"):
        _arrive(opt, base, 2, 4)


def test_chain_plans_every_group_before_launching(monkeypatch):
    """engine.fedopt_chain_ uploads every dtype group's tables before the first launch: a failure
    while planning the second group launches nothing (the kernel is never called)."""
    from flame_amd import _native as N
    launched = []

    real = N.lib()        # (the library loads without a GPU: chunk sizes etc. come from it)

    class FakeLib:
        def flame_fedopt_chain(self, *a):
            launched.append(a[0])
            return 0

        def __getattr__(self, name):
            return getattr(real, name)
    uploads = []

    def upload(meta, device):
        uploads.append(len(meta))
        if len(uploads) == 2:
            raise RuntimeError("out of staging memory")
        return torch.zeros(len(meta), dtype=torch.int64)
    monkeypatch.setattr(N, "lib", lambda: FakeLib())
    monkeypatch.setattr(engine._staging, "upload", upload)
    monkeypatch.setattr(engine, "_client_row", lambda cl, b, dev, keep: ([b.data_ptr()] * len(cl), 0))
    base = [torch.zeros(4096), torch.zeros(4096, dtype=torch.bfloat16)]
    outs = [torch.empty_like(b) for b in base]
    with pytest.raises(RuntimeError, match="out of staging memory"):
        engine.fedopt_chain_("fedadam", base, [None, None], outs, [torch.empty_like(b) for b in base],
                             [torch.empty_like(b) for b in base], [[b] for b in base], [1.0], [True],
                             engine.fedopt_scalars(0.9, 0.99, 1e-2, 1e-3), True, [True, True])
    assert uploads == [uploads[0], uploads[1]] and launched == []
