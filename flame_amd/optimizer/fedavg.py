"""FedAvg on MI355X -- drop-in for lib/python/flame/optimizer/fedavg.py:30-104.

Same contract as the reference: ``base_weights`` is mutated in place and
returned (fedavg.py:74,87); cache entries are consumed with ``cache.pop`` in
``cache.iterkeys()`` order (:79-82); ``rate = count / total`` (:84); ``None``
when the cache is empty or ``total == 0`` (:76-77); extra kwargs such as
``num_trainers`` are accepted and ignored.

The reference's O(N x #tensors) Python loop of two torch ops
(``_aggregate_pytorch``, :89-104) becomes one HIP launch per dtype
(``flame_agg_reduce``) over every key and every client, with the per-element
client order kept sequential so results are bit-identical.

Eager batching (opt-in, ``FedAvg(defer=True)``, e.g. the job config's optimizer
``kwargs``): the eager top aggregator calls ``do()`` once per arrival on the same
``base_weights`` with the running total (``eager_syncfl/top_aggregator.py:36-90``), which
as written reads and writes the whole model per arrival (3 passes of P per update).
Each arrival's rate ``count / total`` is fixed when it arrives, so with ``defer=True``
``do()`` queues it and returns a :class:`DeferredWeights` -- a read-only Mapping over
``base_weights`` -- and the queued arrivals are reduced into ``base_weights`` in ONE
launch, with the identical per-element operation sequence (bit-identical), the moment
anything reads the result (``w[k]``, ``items()``, ``load_state_dict``, ``deepcopy``), a
``do()`` arrives with another base dict, an empty ``do()`` returns ``None``, or
``max_pending`` arrivals / ``max_pending_bytes`` are queued.  ``base_weights`` itself
(a plain dict) lags until then: read the returned object, as flame's roles do.
"""
import collections
import collections.abc
import copy
import logging
import weakref

import torch

from .. import engine, metrics
from .abstract import AbstractOptimizer
from .fedbuff import _own_shm_views
from .regularizer import Regularizer

logger = logging.getLogger(__name__)


class DeferredWeights(collections.abc.Mapping):
    """``base_weights`` plus queued eager arrivals, reduced into it on first read."""

    def __init__(self, base, max_pending, max_pending_bytes=None, owner=None):
        self._base = base
        # the optimizer (weakly: it holds this object; a cycle would keep queued slab slots
        # alive until the cyclic GC): its metric_collector sees the flush's launch
        self._owner = weakref.ref(owner) if owner is not None else None
        self._pending = []         # [(weights, rate)] in arrival order
        self._max_pending = max_pending
        self._max_bytes = max_pending_bytes
        self._held = 0             # bytes of queued arrivals that own their memory (not slab slots)
        self._arrival_bytes = sum(v.numel() * v.element_size() for v in base.values()
                                  if isinstance(v, torch.Tensor))

    def _check(self, w):
        # the reference raises from the do() that brought a bad arrival (fedavg.py:93-104):
        # unknown keys, and `agg += tmp` whose promoted dtype cannot be cast back to the aggregate's
        for k in w.keys():
            if k not in self._base:
                raise KeyError(k)
            acc, dt = self._base[k].dtype, engine.weight_dtype(w, k)
            if dt != acc:
                engine._check_cast(acc, dt)

    def _queue(self, entries):
        for w, _ in entries:
            self._check(w)
        # a view into a sender's shared-memory segment is copied to HBM before do() returns
        entries = [(_own_shm_views(w), r) for w, r in entries]
        self._pending.extend(entries)
        self._held += sum(self._arrival_bytes for w, _ in entries if getattr(w, "slab", None) is None)
        if len(self._pending) >= self._max_pending or (self._max_bytes is not None and self._held > self._max_bytes):
            self.flush()

    @property
    def pending(self):
        return len(self._pending)

    def flush(self):
        """Reduce every queued arrival into ``base_weights`` (one launch per dtype)."""
        if not self._pending:
            return
        entries, self._pending, self._held = self._pending, [], 0
        with metrics.recording(self._owner() if self._owner is not None else None):
            engine.accumulate(self._base, entries)

    def __getitem__(self, k):
        self.flush()
        return self._base[k]

    def __iter__(self):
        return iter(self._base)

    def __len__(self):
        return len(self._base)

    def __contains__(self, k):
        return k in self._base

    def __deepcopy__(self, memo):
        self.flush()
        return copy.deepcopy(self._base, memo)

    def __reduce__(self):
        # pickling (torch.save, a checkpoint) stores the reduced model as a state_dict-style OrderedDict
        return (collections.OrderedDict, (list(self.items()),))

    def materialize(self):
        """``base_weights`` itself, every queued arrival reduced into it."""
        self.flush()
        return self._base


class FedAvg(AbstractOptimizer):
    """FedAvg class."""

    def __init__(self, defer: bool = False, max_pending: int = 256, max_pending_bytes: int = 16 << 30):
        self.agg_weights = None
        self.regularizer = Regularizer()
        self.defer = defer
        self.max_pending = max_pending
        self.max_pending_bytes = max_pending_bytes
        self._deferred = None      # the DeferredWeights the last deferred do() returned

    def _pop_entries(self, cache, total):
        # after popping, the item is removed from the cache (fedavg.py:80-82); rate = count / total
        return [(tres.weights, tres.count / total) for tres in map(cache.pop, list(cache.iterkeys()))]

    def do(self, base_weights, cache, *, total: int = 0, version: int = 0, **kwargs):
        """Aggregate the cached trainer updates into ``base_weights`` (in place)."""
        logger.debug("calling fedavg (flame_amd)")
        assert base_weights is not None
        if isinstance(base_weights, DeferredWeights):
            base_weights = base_weights.materialize()
        pend = self._deferred
        if pend is not None and (pend._base is not base_weights or len(cache) == 0 or total == 0
                                 or not self.defer or "flame_amd_key_groups" in kwargs):
            # another base dict, an empty round or a non-deferred call: the queued arrivals
            # land in their base dict first, as the reference's in-place adds would have
            pend.flush()
            self._deferred = pend = None
        self.agg_weights = base_weights
        if len(cache) == 0 or total == 0:
            return None
        entries = self._pop_entries(cache, total)
        if self.defer and "flame_amd_key_groups" not in kwargs:
            if pend is None:
                self._deferred = pend = DeferredWeights(base_weights, self.max_pending, self.max_pending_bytes,
                                                        owner=self)
            pend._queue(entries)
            return pend
        # flame_amd.shard passes its plan's waves: one launch per wave, its all-gather started
        # right behind it (callers from flame pass no such kwargs)
        engine.accumulate(self.agg_weights, entries, key_groups=kwargs.get("flame_amd_key_groups"),
                          after_group=kwargs.get("flame_amd_after_group"))
        return self.agg_weights
