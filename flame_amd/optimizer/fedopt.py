"""FedOPT family on MI355X -- drop-in for lib/python/flame/optimizer/fedopt.py:33-129.

Control flow is the reference's (fedopt.py:58-92): FedAvg first; ``None`` ->
return ``current_weights``; round 1 -> ``current_weights = agg_weights`` (no
adaptive step); afterwards the adaptive step of ``_adapt_pytorch``
(:102-129) with the subclass's ``_delta_v``.

From the second adaptive-capable round on, fp32 / bf16 / fp16 keys go through
ONE fused kernel per dtype (``flame_fedopt_reduce_adapt``): the client
reduction, ``d``, ``m_t``, ``v_t`` and the new ``current`` are computed in
registers with one rounding per reference op, reading base/cur/m/v once and
writing avg/m/v/cur once, instead of ~12 unfused torch passes.  Other keys
(BatchNorm's int64 ``num_batches_tracked``, which the reference silently
promotes to fp32 in this step, fp64 keys, and any key whose dtype changed) are
reduced by the FedAvg kernel and then run the reference's statements as one
``flame_elementwise`` program per key (``flame_amd.elementwise``: torch's own dtype
promotions, torch-CPU's arithmetic per dtype).

Ownership: ``base_weights`` is mutated in place into the
FedAvg result (``self.agg_weights``); ``m_t``/``v_t`` persist across rounds on
the device; each round returns a NEW OrderedDict of new tensors, like the
reference.  ``d_t`` is not materialised by the fused path; it is computed
lazily from ``agg_weights`` and the previous ``current_weights`` on access.

``defer=True`` (opt-in, like ``FedAvg(defer=True)``) batches the EAGER caller
(eager_syncfl/top_aggregator.py:36-90: one ``do()`` per arrival into the round's base):
each eligible call (fp32 / bf16 / fp16 keys on the GPU) pops its cache entries, queues them and
returns a :class:`DeferredCurrent`; the queue runs as ONE ``flame_fedopt_chain`` launch
when anything reads the results (the returned mapping, ``current_weights``, ``m_t``,
``v_t``, ``agg_weights``), bit-identical to a launch per call.  Until then the base dict
lags, as ``FedAvg(defer=True)``'s does.  ``d_t`` is not kept across a deferred queue.
"""
import collections.abc
import copy
import logging
import os
import weakref
from abc import abstractmethod
from collections import OrderedDict

import torch

from .. import elementwise as ew, engine, metrics
from .fedavg import FedAvg

logger = logging.getLogger(__name__)


def _same_storage(a, b) -> bool:
    return a is b or (a.device == b.device and a.numel() > 0 and a.data_ptr() == b.data_ptr()
                      and a.shape == b.shape and a.stride() == b.stride())


def _byte_range(t):
    end = t.data_ptr() + t.element_size() * (1 + sum((n - 1) * st for n, st in zip(t.shape, t.stride()) if n > 0))
    return t.data_ptr(), end


def _overlaps(a, b) -> bool:
    """Do two tensors' byte ranges intersect?"""
    if a.numel() == 0 or b.numel() == 0:
        return False
    (a0, a1), (b0, b1) = _byte_range(a), _byte_range(b)
    return a0 < b1 and b0 < a1


class FedOPT(FedAvg):
    """FedOPT class."""

    variant = None  # "fedadam" | "fedyogi" | "fedadagrad"
    # two launches per dtype instead of one: the FedAvg reduction (flame_agg_reduce, avg written
    # into base) and then the adaptive step over avg/cur/m/v alone (flame_fedopt_reduce_adapt
    # with no clients) -- bit-identical; which is faster is measured in DESIGN.md §4
    split_launch = os.environ.get("FLAME_AMD_FEDOPT_SPLIT", "0") == "1"

    # deferred eager queue bounds (as FedAvg(defer=True)'s)
    max_chain_entries = 256
    max_chain_bytes = 16 << 30

    def __init__(self, beta_1, beta_2, eta, tau, defer: bool = False):
        self._poisoned = None
        self._chain = None
        self._current = None
        self._m = None
        self._v = None
        self._agg = None
        super().__init__()
        self.chain_defer = defer
        self.current_weights = None
        self._d_t = None
        self._prev_current = None
        self.m_t = None
        self.v_t = None
        self.beta_1 = beta_1
        self.beta_2 = beta_2
        self.eta = eta
        self.tau = tau

    # state the reference keeps as attributes: a read runs whatever eager calls are queued
    @property
    def current_weights(self):
        self._flush_chain()
        return self._current

    @current_weights.setter
    def current_weights(self, value):
        self._flush_chain()
        self._current = value

    @property
    def m_t(self):
        self._flush_chain()
        return self._m

    @m_t.setter
    def m_t(self, value):
        self._flush_chain()
        self._m = value

    @property
    def v_t(self):
        self._flush_chain()
        return self._v

    @v_t.setter
    def v_t(self, value):
        self._flush_chain()
        self._v = value

    @property
    def agg_weights(self):
        self._flush_chain()
        return self._agg

    @agg_weights.setter
    def agg_weights(self, value):
        self._flush_chain()
        self._agg = value

    # d_t is an attribute in the reference; keep it readable (and assignable)
    @property
    def d_t(self):
        if self._d_t is None and self._prev_current is not None and self.agg_weights is not None:
            self._d_t = {k: self.agg_weights[k] - self._prev_current[k] for k in self.agg_weights.keys()}
        return self._d_t

    @d_t.setter
    def d_t(self, value):
        self._d_t = value

    def do(self, base_weights, cache, *, total: int = 0, version: int = 0, **kwargs):
        logger.debug("calling fedopt (flame_amd)")
        self._check_poisoned()
        if self.chain_defer and not kwargs.keys() & _SHARD_KWARGS:
            ch = self._chain
            if ch is not None and ch.base is base_weights and (len(cache) == 0 or total == 0):
                # an arrival with nothing to aggregate: the reference's FedAvg.do returns None
                # and do() hands back current_weights unchanged (fedopt.py:80-85) -- here the
                # queued chain's last result, without cutting the chain; agg_weights reads None
                # once the queue has run, as the reference's self.agg_weights = None (:80-83)
                ch.last_empty = True
                return ch.result(self, len(ch.steps) - 1, list(base_weights.keys()))
            popped = self._try_queue(base_weights, cache, total)
            if isinstance(popped, DeferredCurrent):
                return popped
            if popped is not None:          # not eligible: the popped entries take the normal path
                cache = _Replay(popped)
        self._flush_chain()
        if self.current_weights is not None and base_weights is not None and len(cache) > 0 and total != 0:
            # flame_amd.shard passes its plan's waves (one launch per wave, its all-gather started
            # right behind it) and an allocator placing each key's new `current` straight into
            # the full tensor the gather fills (callers from flame pass none of these)
            return self._do_fused(base_weights, cache, total, kwargs.get("flame_amd_key_groups"),
                                  kwargs.get("flame_amd_after_group"), kwargs.get("flame_amd_out_alloc"))
        self.agg_weights = super().do(base_weights, cache, total=total, version=version)
        if self.agg_weights is None:
            return self.current_weights
        if self.current_weights is None:
            self.current_weights = self.agg_weights
        else:  # pragma: no cover - every non-None path with state goes through _do_fused
            raise AssertionError("unreachable")
        return self.current_weights

    # ------------------------------------------------------------------ fused round
    def _do_fused(self, base_weights, cache, total, key_groups=None, after_group=None, alloc=None):
        self.agg_weights = base_weights
        entries = self._pop_entries(cache, total)
        current = self.current_weights
        device = engine.pick_device(base_weights, current, *[w for w, _ in entries])
        keys = list(base_weights.keys())
        fused, generic = [], []
        float_dts = (torch.float32, torch.bfloat16, torch.float16)
        for k in keys:
            dt = base_weights[k].dtype
            # the eager caller hands the same base dict to every do() of a round, so after the
            # round-1 passthrough current IS base (eager_syncfl/top_aggregator.py:42,75): the
            # reference's d = avg - current is then 0 -- the fused kernel takes cur = avg for such
            # keys (FLAME_SEG_CUR_IS_AVG); only a partial overlap takes the op-sequence path
            aliased = k in current and _same_storage(current[k], base_weights[k])
            partial = (k in current and not aliased and current[k].device == base_weights[k].device
                       and _overlaps(current[k], base_weights[k]))
            ok = (dt in float_dts and k in current and not partial
                  and current[k].dtype == dt and current[k].shape == base_weights[k].shape
                  and all(k in w and w[k].dtype == dt for w, _ in entries)
                  and (self.m_t is None or (k in self.m_t and self.m_t[k].dtype == dt
                                            and self.v_t[k].dtype == dt)))
            (fused if ok else generic).append(k)
        for w, _ in entries:
            for k in w.keys():
                if k not in base_weights:
                    raise KeyError(k)

        state_zero = self.m_t is None
        if state_zero:
            self.m_t, self.v_t = {}, {}
        new_cur = {}
        if generic:       # first, so every key of a group is final when its group is handed on
            sub = {k: base_weights[k] for k in generic}
            engine.accumulate(sub, [({k: w[k] for k in generic if k in w}, r) for w, r in entries], device=device)
            res = self._adapt_generic(generic, base_weights, current, state_zero)
            if alloc is not None:
                for k, v in res.items():
                    res[k] = alloc(k, v.dtype, v.shape).copy_(v)
            new_cur.update(res)
        hyper = engine.fedopt_scalars(self.beta_1, self.beta_2, self.eta, self.tau)
        in_fused = set(fused)
        for gi, group in enumerate(key_groups if key_groups is not None else [keys]):
            ks = [k for k in group if k in in_fused]
            if ks:
                self._launch_fused(ks, base_weights, current, entries, device, hyper, state_zero, alloc, new_cur)
            if after_group is not None:
                after_group(gi)
        self._prev_current = current
        self._d_t = None
        self.current_weights = OrderedDict((k, new_cur[k]) for k in current.keys() if k in new_cur)
        return self.current_weights

    def _launch_fused(self, ks, base_weights, current, entries, device, hyper, state_zero, alloc, new_cur):
        """One flame_fedopt_reduce_adapt launch per dtype over keys ``ks``."""
        targets = [engine._Target(base_weights[k], device) for k in ks]
        alias = [_same_storage(current[k], base_weights[k]) for k in ks]
        # an aliased key's current is the FedAvg result itself: the kernel takes cur = avg
        curs = [t.dev if a else engine._as_device(current[k], device) for t, a, k in zip(targets, alias, ks)]
        outs = [alloc(k, base_weights[k].dtype, base_weights[k].shape) if alloc is not None else
                torch.empty(base_weights[k].shape, dtype=base_weights[k].dtype, device=device) for k in ks]
        ms, vs = [], []
        for k in ks:
            if state_zero:  # zeros_like(d_t[k]) in the reference: d's dtype
                self.m_t[k] = torch.empty(base_weights[k].shape, dtype=base_weights[k].dtype, device=device)
                self.v_t[k] = torch.empty(base_weights[k].shape, dtype=base_weights[k].dtype, device=device)
            else:
                self.m_t[k] = engine._as_device(self.m_t[k], device)
                self.v_t[k] = engine._as_device(self.v_t[k], device)
            ms.append(self.m_t[k])
            vs.append(self.v_t[k])
        avgs = [t.dev for t in targets]
        clients = [[w[k] for w, _ in entries] for k in ks]
        rates = [r for _, r in entries]
        if self.split_launch:
            engine.reduce_(avgs, avgs, clients, rates)
            engine.fedopt_reduce_adapt_(self.variant, [None] * len(ks), avgs, curs, outs, ms, vs,
                                        [[] for _ in ks], [], hyper, state_zero, cur_is_avg=alias)
        else:
            engine.fedopt_reduce_adapt_(self.variant, avgs, avgs, curs, outs, ms, vs, clients, rates, hyper,
                                        state_zero, cur_is_avg=alias)
        for t in targets:
            t.writeback()
        new_cur.update(zip(ks, outs))

    # ------------------------------------------------------------------ deferred eager chain
    def _try_queue(self, base_weights, cache, total):
        """Queue an eager do() call if it can run on flame_fedopt_chain; returns the
        DeferredCurrent, or the popped (key, TrainResult) pairs when the call is not eligible
        (None if nothing was popped)."""
        if self._current is None and self._chain is None:
            return None                      # round 1: the passthrough, not an adaptive step
        if base_weights is None or len(cache) == 0 or total == 0:
            return None
        if not _chain_tensors(base_weights):
            return None
        ch = self._chain
        if ch is not None and (ch.base is not base_weights or ch.n_entries >= self.max_chain_entries
                               or ch.nbytes >= self.max_chain_bytes):
            self._flush_chain()
            ch = None
        popped = [(k, cache.pop(k)) for k in list(cache.iterkeys())]
        keys = list(base_weights.keys())
        shapes = {k: base_weights[k].shape for k in keys}
        device = base_weights[keys[0]].device
        for _, tres in popped:
            w = tres.weights
            # an update the per-call path would refuse (wrong size) is not queued: it raises from
            # its own do() there (slab slots are strided (tiles, T) views of the key)
            if set(w.keys()) != set(keys) or not all(
                    w[k].dtype == base_weights[k].dtype and w[k].device == device
                    and (w[k].numel() == base_weights[k].numel()
                         or engine.tiled_stride(w[k], base_weights[k].numel()))
                    for k in keys):
                self._flush_chain()
                return popped
        if ch is None:
            cur = self._current
            if cur is None or list(cur.keys()) != keys:
                return popped
            aliased = {}
            for k in keys:
                c, b = cur[k], base_weights[k]
                if not (isinstance(c, torch.Tensor) and c.dtype == b.dtype and c.shape == b.shape
                        and c.device == device and c.is_contiguous()):
                    return popped
                aliased[k] = _same_storage(c, b)
                if not aliased[k] and _overlaps(c, b):
                    return popped
            if self._m is not None and not all(
                    k in self._m and k in self._v and self._m[k].dtype == base_weights[k].dtype
                    and self._v[k].dtype == base_weights[k].dtype and self._m[k].shape == shapes[k]
                    and self._m[k].device == device and self._v[k].device == device
                    and self._m[k].is_contiguous() and self._v[k].is_contiguous() for k in keys):
                return popped
            ch = self._chain = _Chain(base_weights, cur, aliased, self._m is None)
        step = [(tres.weights, tres.count / total) for _, tres in popped]
        ch.last_empty = False
        ch.steps.append(step)
        ch.n_entries += len(step)
        ch.nbytes += len(step) * sum(base_weights[k].numel() * 4 for k in keys)
        ch.results.append([])
        return ch.result(self, len(ch.steps) - 1, keys)

    def _flush_chain(self):
        """Run the queued eager calls (if any): one flame_fedopt_chain launch per stretch that
        ends at a still-referenced DeferredCurrent (normally just the last one)."""
        ch = self.__dict__.get("_chain")
        if ch is None:
            return
        self._check_poisoned()
        self._chain = None
        last = len(ch.steps) - 1
        cuts = sorted({i for i, refs in enumerate(ch.results) if any(r() is not None for r in refs)} | {last})
        keys = list(ch.base.keys())
        hyper = engine.fedopt_scalars(self.beta_1, self.beta_2, self.eta, self.tau)
        with metrics.recording(self):      # a queue run at a read is reported like do()'s launches
            self._run_chain(ch, cuts, keys, hyper)

    def _run_chain(self, ch, cuts, keys, hyper):
        """One flame_fedopt_chain launch per stretch of queued calls (one per dtype group; every
        group is planned and uploaded before the first launches, engine.fedopt_chain_).  The
        optimizer's state (m_t / v_t, current_weights, agg_weights) moves to a stretch's results
        only once its launches have returned; if a stretch fails before any of its launches ran,
        the state stays at the last stretch that ran and every result of the stretches that did
        not run re-raises the failure when read.  If a later dtype group's launch fails after an
        earlier group's ran (the exception carries ``flame_partial``), base / m / v no longer
        agree across keys: the optimizer is poisoned and every later call raises."""
        cur, aliased, zero, start = ch.current, ch.aliased, ch.state_zero, 0
        try:
            for cut in cuts:
                steps = ch.steps[start:cut + 1]
                base = [ch.base[k] for k in keys]
                m = {k: torch.empty_like(ch.base[k]) for k in keys} if zero else self._m
                v = {k: torch.empty_like(ch.base[k]) for k in keys} if zero else self._v
                outs = [torch.empty_like(ch.base[k]) for k in keys]
                ends = [j == len(st) - 1 for st in steps for j in range(len(st))]
                engine.fedopt_chain_(self.variant, base, [None if aliased[k] else cur[k] for k in keys], outs,
                                     [m[k] for k in keys], [v[k] for k in keys],
                                     [[w[k] for st in steps for w, _ in st] for k in keys],
                                     [r for st in steps for _, r in st], ends, hyper, zero,
                                     [aliased[k] for k in keys])
                new = OrderedDict(zip(keys, outs))
                self._m, self._v, self._current, self._agg = m, v, new, ch.base
                self._prev_current = None      # d_t is not kept across a deferred queue
                self._d_t = None
                for ref in ch.results[cut]:
                    r = ref()
                    if r is not None:
                        r._value = new
                cur, aliased, zero, start = new, {k: False for k in keys}, False, cut + 1
            if ch.last_empty:        # the last queued call had nothing to aggregate (fedopt.py:80-85)
                self._agg = None
        except BaseException as e:
            if getattr(e, "flame_partial", False):
                # one dtype group's launch ran, a later one's failed: base / m / v of the first
                # group moved on, the others did not -- no later call may reuse that state
                self._poisoned = e
            for refs in ch.results[start:]:
                for ref in refs:
                    r = ref()
                    if r is not None and r._value is None:
                        r._error = e
            raise
        finally:
            # the queued updates (slab slots among them) are released now, not when the last
            # DeferredCurrent dies (the role keeps that one as its weights)
            ch.steps, ch.current, ch.base = [], None, None

    def _check_poisoned(self):
        e = self.__dict__.get("_poisoned")
        if e is not None:
            raise RuntimeError("flame_amd FedOPT: a queued round's launch failed after part of the model's dtype "
                               "groups had been updated, so m_t / v_t / current_weights no longer agree; "
                               f"re-create the optimizer ({type(e).__name__}: {e})") from e

    def _adapt_generic(self, keys, average, current, state_zero):
        """fedopt.py:106-129 for the keys the fused kernel does not take (int buffers such as
        num_batches_tracked, mixed-dtype and fp64 keys): the reference's statements, the
        subclass's _delta_v_tensor included, recorded on elementwise.Lazy operands and run as
        ONE flame_elementwise launch per key -- torch's own dtype promotions, torch-CPU's
        arithmetic per dtype (include/flame_amd.h), no PyTorch compute."""
        out = {}
        programs = self.__dict__.setdefault("_ew_programs", {})
        hyper = (self.beta_1, self.beta_2, self.eta, self.tau)
        groups = {}
        for k in keys:
            ins = [average[k], current[k]]
            if not (state_zero or k not in self.m_t or k not in self.v_t):
                ins += [self.m_t[k], self.v_t[k]]
            # one compiled program per dtype / 0-dim signature, one launch per program and device:
            # a ResNet's BatchNorm num_batches_tracked keys all share one
            sig = (hyper, tuple((t.dtype, t.dim() == 0) for t in ins))
            if sig not in programs:
                programs[sig] = ew.trace(self._adapt_statement, [(t.dtype, tuple(t.shape)) for t in ins])
            groups.setdefault((sig, average[k].device), []).append((k, ins))
        for (sig, device), rows in groups.items():
            res = programs[sig].run_many([ins for _, ins in rows], device)
            for (k, _), (m, v, new) in zip(rows, res):
                self.m_t[k], self.v_t[k], out[k] = m, v, new
        return out

    def _adapt_statement(self, avg, cur, m=None, v=None):
        """fedopt.py:106-129 on Lazy operands (m / v None: the first adaptive round's zeros)."""
        d = avg - cur
        m = torch.zeros_like(d) if m is None else m
        m = self.beta_1 * m + (1 - self.beta_1) * d
        v = torch.zeros_like(d) if v is None else v
        v = self._delta_v_tensor(v, d)
        return m, v, cur + self.eta * m / (torch.sqrt(v) + self.tau)

    @abstractmethod
    def _delta_v_tensor(self, v, d):
        """The subclass's _delta_v_pytorch for one key."""


_SHARD_KWARGS = {"flame_amd_key_groups", "flame_amd_after_group", "flame_amd_out_alloc"}


_CHAIN_DTYPES = (torch.float32, torch.bfloat16, torch.float16)


def _chain_tensors(weights) -> bool:
    """A base dict flame_fedopt_chain can update in place: fp32 / bf16 / fp16, contiguous, one GPU."""
    try:
        ts = list(weights.values())
    except AttributeError:
        return False
    if not ts or not all(isinstance(t, torch.Tensor) for t in ts):
        return False
    dev = ts[0].device
    return dev.type == "cuda" and all(t.dtype in _CHAIN_DTYPES and t.is_contiguous() and t.device == dev for t in ts)


class _Chain:
    """Eager do() calls queued for one flame_fedopt_chain launch."""

    def __init__(self, base, current, aliased, state_zero):
        self.base = base                # the round's base dict (updated in place at the flush)
        self.current = current          # current_weights when the queue started
        self.aliased = aliased          # {key: current[key] IS base[key]} (right after the passthrough)
        self.state_zero = state_zero    # m_t / v_t were None
        self.steps = []                 # per do(): [(weights, rate), ...]
        self.results = []               # per do(): weakrefs to the DeferredCurrents handed out for it
        self.n_entries = 0
        self.nbytes = 0
        self.last_empty = False         # the last do() call queued had nothing to aggregate

    def result(self, owner, step, keys):
        res = DeferredCurrent(owner, self, step, keys)
        self.results[step].append(weakref.ref(res))
        return res


class _Replay:
    """Popped cache entries handed back to the non-deferred path, in the same order."""

    def __init__(self, popped):
        self._items = list(popped)

    def __len__(self):
        return len(self._items)

    def iterkeys(self):
        return iter([k for k, _ in self._items])

    def pop(self, key, default=None):
        for i, (k, v) in enumerate(self._items):
            if k == key:
                del self._items[i]
                return v
        return default


class DeferredCurrent(collections.abc.Mapping):
    """The ``current_weights`` a deferred eager ``do()`` returns (the reference returns a new
    OrderedDict per call): the queued calls up to and including this one run on first read."""

    def __init__(self, owner, chain, step, keys):
        self._owner, self._chain, self._step, self._keys = owner, chain, step, keys
        self._value = None
        self._error = None

    def materialize(self):
        if self._value is None and self._error is None:
            self._owner._flush_chain()
        if self._error is not None:
            raise RuntimeError("the queued FedOPT do() call this result belongs to did not run: "
                               f"{type(self._error).__name__}: {self._error}") from self._error
        return self._value

    def __getitem__(self, k):
        return self.materialize()[k]

    def __iter__(self):
        return iter(self._keys)

    def __len__(self):
        return len(self._keys)

    def __contains__(self, k):
        return k in self._keys

    def __deepcopy__(self, memo):
        return copy.deepcopy(self.materialize(), memo)

    def __reduce__(self):
        return (OrderedDict, (list(self.materialize().items()),))
