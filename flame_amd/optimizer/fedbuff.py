"""FedBuff on MI355X -- drop-in for lib/python/flame/optimizer/fedbuff.py:38-157.

Same contract: ``rate = 1/math.sqrt(1 + version - tres.version)`` computed in
Python (so stale-version errors raise exactly as in the reference, :96); with
``agg_goal_weights is None`` each cached entry re-creates the aggregate
(:139-140,154-155), so only the last entry of that call survives (reference
quirk, kept); otherwise ``agg[k] += tmp`` in place.  ``scale_add_agg_weights``
mutates and returns ``base_weights`` (:122-127); integer tensors raise like
torch's ``int += float`` does.

Batching (MI355X-native, on by default): the async callers hand FedBuff ONE
arrival per ``do()`` (asyncfl/top_aggregator.py:85-92), which as written costs
an accumulator read+write per arrival (3 passes of P per update).  With
``defer=True`` ``do()`` returns a :class:`DeferredAggregate` -- a read-only
Mapping over the same keys -- and queues the arrival; the queued arrivals are
reduced in ONE launch, in arrival order with the identical per-element
operation sequence (bit-identical), the moment anything reads the aggregate
(``agg[k]``, iteration with values, ``scale_add_agg_weights``, ``deepcopy``) or
``max_pending`` arrivals are queued.  ``defer=False`` restores one launch per
``do()`` and a plain dict.
"""
import collections
import collections.abc
import copy
import itertools
import logging
import math
import weakref

import numpy as np
import torch

from .. import engine, metrics, shm_lease
from .abstract import AbstractOptimizer
from .regularizer import Regularizer

logger = logging.getLogger(__name__)


class DeferredAggregate(collections.abc.Mapping):
    """FedBuff aggregate whose queued arrivals are reduced on first read."""

    def __init__(self, weights, max_pending, max_pending_bytes=None, owner=None):
        # the optimizer (weakly: it holds this object; a cycle would keep queued slab slots
        # alive until the cyclic GC): its metric_collector sees the flush's launches
        self._owner = weakref.ref(owner) if owner is not None else None
        self._slabs_ok = weakref.WeakSet()   # slabs whose slots passed _queue's key / dtype checks (weak: a
                                             # replaced cache must not keep its multi-GB slab alive)
        self._keys = list(weights.keys())
        self._meta = {k: (engine.logical_shape(weights, k), engine.weight_dtype(weights, k)) for k in self._keys}
        self._data = None          # dict of device tensors once materialised
        self._pending = []         # [(weights, rate)] in arrival order
        # while every queued arrival is a whole slot of ONE slab: that slab and the slots in
        # queue order (pointer rows then come from slot numbers, no per-arrival pass); None =
        # nothing queued, False = mixed
        self._pend_slab = None
        self._pend_slots = []
        self._max_pending = max_pending
        self._max_bytes = max_pending_bytes
        self._held = 0             # bytes of queued arrivals that own their memory (not slab slots)
        self._arrival_bytes = sum(math.prod(s) * dt.itemsize
                                  for s, dt in self._meta.values())

    def _queue(self, entries):
        held = 0
        last_ok = None                # the slab whose slots the previous entry was checked against
        ps, slots = self._pend_slab, []   # committed with the entries (a KeyError leaves both as they were)
        for w, _ in entries:
            slab = getattr(w, "slab", None)
            if slab is None:
                # a queued arrival keeps its update alive (the reference frees it once folded
                # in); slab slots are preallocated, anything else counts against max_pending_bytes
                held += self._arrival_bytes
            whole_slot = slab is not None and getattr(w, "ranges", None) is None
            if not (whole_slot and (slab is last_ok or slab in self._slabs_ok)):
                for k in w.keys():    # (the slots of one slab share keys and dtypes: checked once)
                    if k not in self._meta:
                        raise KeyError(k)
                    # `agg[k] += tmp` (fedbuff.py:157) raises from the do() that brings it
                    dt = engine.weight_dtype(w, k)
                    if dt != self._meta[k][1]:
                        engine._check_cast(self._meta[k][1], dt)
                if whole_slot:
                    self._slabs_ok.add(slab)
            if whole_slot:
                last_ok = slab
                if ps is None or ps is slab:
                    ps = slab
                    slots.append(w.slot)
                else:
                    ps = False
            else:
                ps = False
        # an arrival decoded in place from a sender's shared-memory segment is copied to HBM
        # before do() returns: the sender may rewrite the segment while it waits in the queue
        if shm_lease.active():
            entries = [(_own_shm_views(w), r) for w, r in entries]
        self._pending.extend(entries)
        self._pend_slab = ps
        if ps:
            self._pend_slots.extend(slots)
        self._held += held
        if len(self._pending) >= self._max_pending or (self._max_bytes is not None and self._held > self._max_bytes):
            self.flush()

    def flush(self):
        """Reduce every queued arrival (one launch per dtype)."""
        if not self._pending:
            return
        with metrics.recording(self._owner() if self._owner is not None else None):
            self._flush()

    def _flush(self):
        if self._data is None and not _uniform(self):
            # later arrivals carry a subset of the first one's keys, or other dtypes: the
            # reference adds them key by key (fedbuff.py:143-157), so does accumulate()
            (w0, r0), rest = self._pending[0], self._pending[1:]
            self._data = collections.OrderedDict(engine.first_tmp(w0, r0))
            if rest:
                engine.accumulate(self._data, rest)
        elif self._data is None:
            # None-start: agg = tmp(first) (fedbuff.py:139-140,154-155), then += the rest
            device = engine.pick_device(*[w for w, _ in self._pending])
            self._data = collections.OrderedDict(
                (k, torch.empty(self._meta[k][0], dtype=self._meta[k][1], device=device)) for k in self._keys)
            engine.reduce_([self._data[k] for k in self._keys], None,
                           [[w[k] for w, _ in self._pending] for k in self._keys],
                           [r for _, r in self._pending], init_first=True)
        else:
            engine.accumulate(self._data, self._pending)
        self._clear_pending()

    def _clear_pending(self):
        self._pending = []
        self._pend_slab = None
        self._pend_slots = []
        self._held = 0

    def __getitem__(self, k):
        self.flush()
        return self._data[k]

    def __iter__(self):
        return iter(self._keys)

    def __len__(self):
        return len(self._keys)

    def __deepcopy__(self, memo):
        self.flush()
        return copy.deepcopy(dict(self._data), memo)

    def __reduce__(self):
        # pickling (torch.save, a checkpoint) stores the reduced aggregate as a state_dict-style OrderedDict
        self.flush()
        return (collections.OrderedDict, (list(self._data.items()),))

    def materialize(self):
        """The aggregate as a plain dict of tensors (flushes)."""
        self.flush()
        return dict(self._data)


def _own_shm_views(weights):
    """``weights`` with every tensor that aliases a sender's shared-memory segment copied to
    the device (synchronously); the dict itself when there is none."""
    if not shm_lease.active() or getattr(weights, "slab", None) is not None:
        return weights            # no segment open, or a slab slot (device memory)
    hit = [k for k, v in weights.items() if isinstance(v, torch.Tensor) and shm_lease.aliases(v)]
    if not hit:
        return weights
    device = engine.pick_device()
    out = collections.OrderedDict()
    for k, v in weights.items():
        if k in hit:
            shm_lease.check_live(v)
            v = v.to(device, non_blocking=False)
        out[k] = v
    return out


class FedBuff(AbstractOptimizer):
    """FedBuff class."""

    def __init__(self, defer: bool = True, max_pending: int = 256, fuse_scale_add: bool = True,
                 max_pending_bytes: int = 16 << 30):
        self.agg_goal_weights = None
        self.is_agg_weights_none = True
        self.regularizer = Regularizer()
        self.defer = defer
        self.max_pending = max_pending
        self.max_pending_bytes = max_pending_bytes
        self.fuse_scale_add = fuse_scale_add

    def do(self, agg_goal_weights, cache, *, total: int = 0, version: int = 0, **kwargs):
        logger.debug("calling fedbuff (flame_amd)")
        self.agg_goal_weights = agg_goal_weights
        self.is_agg_weights_none = self.agg_goal_weights is None
        if len(cache) == 0 or total == 0:
            return None
        entries = []
        try:
            for k in list(cache.iterkeys()):
                tres = cache.pop(k)
                # rate determined based on the staleness of local model (fedbuff.py:94-96)
                rate = 1 / math.sqrt(1 + version - tres.version)
                entries.append((tres.weights, rate))
        finally:
            self._apply(entries)  # what the reference had applied before any exception
        return self.agg_goal_weights

    def do_arrivals(self, agg_goal_weights, arrivals, *, version: int = 0):
        """Several arrivals in ONE call -- the batched form of the async roles' loop.

        Identical to running, for each ``TrainResult`` in ``arrivals`` (arrival order), what
        ``asyncfl/middle_aggregator.py:190-203`` / ``asyncfl/top_aggregator.py:85-92`` do per
        received message: ``cache[end] = tres; agg = self.do(agg, cache, total=tres.count,
        version=version)``.  Same staleness rate per arrival (``1 / math.sqrt(1 + version -
        tres.version)``, fedbuff.py:94-96 -- numpy's IEEE sqrt and division give the same
        doubles), the same None-start (the first arrival starts a None aggregate, the rest add
        to it), and the same error at the same arrival: the arrivals before a stale-version one
        are applied, then ``ZeroDivisionError`` / ``ValueError`` is raised as by ``math``.
        Arrivals with ``count <= 0`` are refused (``ValueError``): the roles never hand them to
        ``do()`` (``if weights is not None and count > 0``, :196).  Returns the aggregate (a
        :class:`DeferredAggregate` with ``defer=True``: the arrivals join its queue at once).
        """
        arrivals = list(arrivals)
        if not arrivals:
            return agg_goal_weights
        n = len(arrivals)
        if any(t.count <= 0 for t in arrivals):
            raise ValueError("FedBuff.do_arrivals: an arrival with count <= 0 (the roles skip those)")
        d = 1 + version - np.fromiter((t.version for t in arrivals), dtype=np.int64, count=n)
        bad = np.flatnonzero(d <= 0)
        upto = int(bad[0]) if bad.size else n
        rates = (1.0 / np.sqrt(d[:upto].astype(np.float64))).tolist()
        entries = [(t.weights, r) for t, r in zip(arrivals, rates)]
        self.agg_goal_weights = agg_goal_weights
        self.is_agg_weights_none = agg_goal_weights is None
        if entries and self.is_agg_weights_none:
            self._apply(entries[:1])          # the first arrival's do(): a None-start
            entries = entries[1:]
            self.is_agg_weights_none = not entries
        self._apply(entries)                  # every later do() adds to the aggregate
        if upto < n:
            math.sqrt(int(d[upto]))           # raises ValueError (math domain error) when negative
            raise ZeroDivisionError("float division by zero")
        return self.agg_goal_weights

    def _apply(self, entries):
        if not entries:
            return
        if self.is_agg_weights_none:
            # each cached entry re-creates the aggregate: only the last one survives (fedbuff.py:139-140)
            weights, rate = entries[-1]
            if self.defer:
                agg = DeferredAggregate(weights, self.max_pending, self.max_pending_bytes, owner=self)
                agg._queue([(weights, rate)])
                self.agg_goal_weights = agg
            else:
                self.agg_goal_weights = engine.first_tmp(weights, rate)
        elif isinstance(self.agg_goal_weights, DeferredAggregate):
            self.agg_goal_weights._queue(entries)
        else:
            engine.accumulate(self.agg_goal_weights, entries)

    def scale_add_agg_weights(self, base_weights, agg_goal_weights, agg_goal: int, **kwargs):
        """base[k] += agg[k] / agg_goal in place; returns base_weights (fedbuff.py:101-127).
        flame_amd.shard passes its waves (``flame_amd_key_groups`` / ``flame_amd_after_group``:
        one launch per wave, its all-gather started behind it); flame passes none."""
        return self._scale_add(base_weights, agg_goal_weights, agg_goal, None,
                               kwargs.get("flame_amd_key_groups"), kwargs.get("flame_amd_after_group"))

    def scale_add_agg_weights_with_delta(self, base_weights, agg_goal_weights, agg_goal: int):
        """scale_add fused with the middle aggregator's upload delta (new - old).

        Equals ``prev = deepcopy(w); scale_add(w, ...); delta_weights_pytorch(w, prev)``
        (asyncfl/middle_aggregator.py:221-226,246; common/util.py:152-159) in one pass.
        Returns ``(base_weights, delta)``.
        """
        device = engine.pick_device(base_weights, agg_goal_weights)
        delta = {k: torch.empty(base_weights[k].shape, dtype=base_weights[k].dtype, device=device)
                 for k in base_weights.keys()}
        return self._scale_add(base_weights, agg_goal_weights, agg_goal, delta), delta

    def _scale_add(self, base_weights, agg_goal_weights, agg_goal, delta, key_groups=None, after_group=None):
        if isinstance(agg_goal_weights, DeferredAggregate):
            if self.fuse_scale_add and _fused_scale_add(base_weights, agg_goal_weights, agg_goal, delta, key_groups,
                                                        after_group):
                return base_weights
            agg_goal_weights.flush()
        device = engine.pick_device(base_weights, agg_goal_weights)
        for gi, keys in enumerate(key_groups if key_groups is not None else [list(base_weights.keys())]):
            targets = [engine._Target(base_weights[k], device) for k in keys]
            engine.scale_add_([t.dev for t in targets], [agg_goal_weights[k] for k in keys], agg_goal,
                              [delta[k] for k in keys] if delta is not None else None)
            for t in targets:
                t.writeback()
            if after_group is not None:
                after_group(gi)
        return base_weights


def _fused_scale_add(base_weights, agg, agg_goal, delta, key_groups=None, after_group=None) -> bool:
    """``base += agg / agg_goal`` (+ the delta) straight from a None-start aggregate whose
    arrivals are still queued: the arrivals are reduced in registers and applied in ONE
    ``flame_hier_fedbuff`` launch per dtype (one middle, no top) -- the aggregate is never
    written to HBM and read back (asyncfl/top_aggregator.py:85-110: the top queues its
    aggGoal arrivals, then scale_adds once).  Bit-identical to flush + scale_add: the same
    op per element.  The aggregate stays readable (its arrivals stay queued and are reduced
    if anything reads it).  Returns False (nothing done) when the case does not apply."""
    if agg._data is not None or not agg._pending or not agg_goal or not _uniform(agg):
        return False
    keys = list(base_weights.keys())
    if keys != agg._keys:
        return False
    device = engine.pick_device(base_weights, *[w for w, _ in agg._pending])
    codes = {}
    for k in keys:
        t = base_weights[k]
        shape, dt = agg._meta[k]
        code = engine.DTYPE_CODE.get(dt)
        if (code not in (engine.N.FLAME_F32, engine.N.FLAME_BF16, engine.N.FLAME_F16) or t.dtype != dt
                or t.device != device or not t.is_contiguous() or t.numel() != math.prod(shape)
                or (delta is not None and (delta[k].device != device or not delta[k].is_contiguous()))):
            return False
        codes[k] = code
    rows, keep = _hier_rows([agg], keys, device)
    if rows is None:
        return False
    rates = [[r for _, r in agg._pending]]
    for gi, gkeys in enumerate(key_groups if key_groups is not None else [keys]):
        groups = collections.OrderedDict()
        for k in gkeys:
            groups.setdefault(codes[k], []).append(k)
        for code, ks in groups.items():
            segs = [engine.HierSeg(numel=base_weights[k].numel(), mid_w=[base_weights[k].data_ptr()],
                                   clients=rows[k][0], mid_delta=[delta[k].data_ptr()] if delta is not None else None,
                                   tile_stride=rows[k][1]) for k in ks]
            engine.hier_fedbuff_(segs, code, rates, [agg_goal], [1.0], top_accum=False, top_goal=None, device=device,
                                 keep=keep)
        if after_group is not None:
            after_group(gi)
    engine._keepalive(keep, device)
    return True


# ---------------------------------------------------------------- co-located middle aggregators
def _uniform(agg: DeferredAggregate) -> bool:
    """Every queued arrival carries every key in the aggregate's dtype, a dtype the kernels
    carry (the one-launch case)."""
    slab = agg._pend_slab
    if slab:        # every arrival a whole slot of one slab: its keys / dtypes decide for all
        return (len(slab.keys) == len(agg._keys)
                and all(k in slab.meta and slab.meta[k][0] == dt and dt in engine.DTYPE_CODE
                        for k, (_, dt) in agg._meta.items()))
    return all(agg._meta[k][1] in engine.DTYPE_CODE for k in agg._keys) and all(k in w and engine.weight_dtype(w, k) == agg._meta[k][1]
               for w in engine.representatives([w for w, _ in agg._pending]) for k in agg._keys)


def flush_aggregates(aggs):
    """Reduce the queued arrivals of several independent FedBuff aggregates at once.

    For middle aggregators that share a GPU (LIFL-style hierarchies,
    asyncfl/middle_aggregator.py:164-256): every aggregate keeps its own arrival
    order and staleness rates (FLAME_AGG_SEG_RATES gives each segment its own
    rate row), so the result is bit-identical to flushing them one by one, but
    all aggregates with the same number of queued arrivals and the same start
    (None-start or accumulate) go in one launch per dtype.
    """
    groups = collections.OrderedDict()
    for a in aggs:
        if not isinstance(a, DeferredAggregate) or not a._pending:
            continue
        if not _uniform(a):
            a.flush()
            continue
        groups.setdefault((a._data is None, len(a._pending)), []).append(a)
    for (init, _), members in groups.items():
        if len(members) == 1:
            members[0].flush()
            continue
        device = engine.pick_device(*[w for a in members for w, _ in a._pending])
        outs, clients, rows = [], [], []
        for a in members:
            if init:
                a._data = collections.OrderedDict(
                    (k, torch.empty(a._meta[k][0], dtype=a._meta[k][1], device=device)) for k in a._keys)
            row = [r for _, r in a._pending]
            for k in a._keys:
                outs.append(a._data[k])
                clients.append([w[k] for w, _ in a._pending])
                rows.append(row)
        engine.reduce_(outs, None if init else outs, clients, None, init_first=init, seg_rates=rows)
        for a in members:
            a._clear_pending()


def scale_add_many(pairs, agg_goal: int, with_delta: bool = False):
    """``scale_add_agg_weights`` (optionally fused with the middle's delta) for several
    (base_weights, agg_goal_weights) pairs in one launch per dtype; bit-identical to
    calling it pair by pair.  Returns the list of base_weights (or of (base, delta))."""
    flush_aggregates([agg for _, agg in pairs])
    device = engine.pick_device(*[b for b, _ in pairs], *[a for _, a in pairs])
    targets, aggs, deltas, results = [], [], [], []
    for base, agg in pairs:
        delta = None
        if with_delta:
            delta = {k: torch.empty(base[k].shape, dtype=base[k].dtype, device=device) for k in base.keys()}
        for k in base.keys():
            targets.append(engine._Target(base[k], device))
            aggs.append(agg[k])
            if delta is not None:
                deltas.append(delta[k])
        results.append((base, delta) if with_delta else base)
    engine.scale_add_([t.dev for t in targets], aggs, agg_goal, deltas if with_delta else None)
    for t in targets:
        t.writeback()
    return results


# ---------------------------------------------------------------- co-located hierarchy, one pass
class _OneEntryCache(dict):
    def iterkeys(self):
        return iter(list(self.keys()))


def _compose_hierarchy(middles, top_agg, version, top_weights, top_goal, with_delta, update_middle_weights=True):
    """The reference's op sequence with the separate launches (fallback of hierarchy_round)."""
    from .train_result import TrainResult
    top = FedBuff(fuse_scale_add=False)     # the separate launches, as the roles issue them
    deltas = []
    for w, agg, goal, mv in middles:
        lw = {k: engine.logical_tensor(w, k) for k in w.keys()}
        tiled = [k for k in lw if lw[k] is not w[k]]       # slab-slot middles: work on logical copies
        if not update_middle_weights or tiled:
            lw = {k: v.clone() for k, v in lw.items()}
        _, d = FedBuff(fuse_scale_add=False).scale_add_agg_weights_with_delta(lw, agg, goal)
        if update_middle_weights:
            for k in tiled:
                _write_tiled(w[k], lw[k])
        deltas.append(d)
        cache = _OneEntryCache(mid=TrainResult(d, 1, mv))
        top_agg = top.do(top_agg, cache, total=1, version=version)
    if top_weights is not None:
        top.scale_add_agg_weights(top_weights, top_agg, top_goal)
    return top_agg, (deltas if with_delta else None)


def _write_tiled(view, logical):
    """Store a logical tensor back into its tiled slab view (padding past numel zeroed)."""
    flat = torch.zeros(view.numel(), dtype=view.dtype, device=view.device)
    flat[:logical.numel()] = logical.reshape(-1)
    view.copy_(flat.view(view.shape))


def _tiled_stride(ts, n):
    """0 if every tensor is a contiguous n-element tensor; the common tile stride (bytes) if
    every one is a tiled slab view of n logical elements with one shape; else None."""
    st = {engine.tiled_stride(t, n) if t.is_cuda else 0 for t in ts}
    if st == {0}:
        return 0 if all(t.is_contiguous() and t.numel() == n for t in ts) else None
    if len(st) == 1 and len({tuple(t.shape) for t in ts}) == 1:
        return st.pop()
    return None


def _hier_rows(aggs, keys, device):
    """Per key: (arrival pointers middle-major, tile stride), or None if no single stride fits."""
    meta = aggs[0]._meta
    slab = aggs[0]._pend_slab
    if slab and all(a._pend_slab is slab for a in aggs):
        # every arrival of every middle is a whole slot of one slab (tracked as they queued)
        slots = np.fromiter(itertools.chain.from_iterable(a._pend_slots for a in aggs), dtype=np.uint64)
        rows = engine.slot_rows(slab, None, slots, keys, {k: math.prod(meta[k][0]) for k in keys},
                                {k: meta[k][1] for k in keys}, device)
        if rows is not None:
            return rows, []
    rows = engine.slab_rows([w for a in aggs for w, _ in a._pending], keys,
                            {k: math.prod(meta[k][0]) for k in keys}, {k: meta[k][1] for k in keys}, device)
    if rows is not None:
        return rows, []
    rows, keep = {}, []
    for k in keys:
        shape, dt = aggs[0]._meta[k]
        ref = torch.empty(shape, dtype=dt, device="meta")   # numel / dtype of the aggregate
        ptrs, stride = [], None
        for a in aggs:
            row, ts = engine._client_row([w[k] for w, _ in a._pending], ref, device, keep)
            if stride is None:
                stride = ts
            elif ts != stride:
                return None, keep
            ptrs.extend(row)
        rows[k] = (np.asarray(ptrs, dtype=np.uint64), stride)
    return rows, keep


def hierarchy_round(middles, top_agg=None, *, version: int, top_weights=None, top_goal=None,
                    with_delta: bool = False, update_middle_weights: bool = True, key_groups=None, after_group=None):
    """A node's co-located two-level FedBuff hierarchy in ONE pass per dtype.

    ``middles``: sequence of ``(mid_weights, mid_agg, mid_goal, mid_version)`` in the order
    the top aggregator receives their deltas.  ``mid_agg`` is the middle's FedBuff aggregate
    (normally the :class:`DeferredAggregate` its ``do()`` calls returned).  Equivalent to,
    for each middle: ``scale_add_agg_weights_with_delta(mid_weights, mid_agg, mid_goal)``
    (fedbuff.py:101-127 + asyncfl/middle_aggregator.py:221-226,246), then the top's
    ``top_agg = FedBuff.do(top_agg, {delta, version=mid_version}, version=version)``
    (asyncfl/top_aggregator.py:85-92, rate 1/sqrt(1+version-mid_version), fedbuff.py:96);
    finally, if ``top_weights`` is given, ``scale_add_agg_weights(top_weights, top_agg,
    top_goal)``.  Bit-identical to that sequence; the middle aggregates and (unless
    ``with_delta``) the deltas never reach HBM.  Middle weights and ``top_weights`` are
    updated in place.  Returns ``(top_agg, deltas or None)``.

    The middle aggregates stay valid: their queued arrivals are kept and reduced again
    if anything reads them later.

    ``update_middle_weights=False`` leaves the middles' weights untouched (nothing is
    written back; the same tensor may then serve several middles).  That is the async
    hierarchy as the reference composes it: a middle's updated weights only feed its
    upload delta (asyncfl/middle_aggregator.py:244-246) and are replaced by the top's
    model at its next fetch (:119-120) -- here the delta goes straight to the top.

    ``key_groups`` / ``after_group``: as for ``engine.accumulate`` -- one launch per dtype
    per group of keys, ``after_group(i)`` called once group ``i`` is queued (the sharded
    hierarchy all-gathers the top model's pieces of that group there).
    """
    middles = list(middles)
    if not middles:
        raise ValueError("hierarchy_round: no middles")
    if top_weights is not None and not top_goal:
        raise ValueError("hierarchy_round: top_goal must be nonzero")
    # the top's rates, computed as FedBuff.do does (stale versions raise here, fedbuff.py:96)
    top_rates = [1 / math.sqrt(1 + version - mv) for *_, mv in middles]
    aggs = [a for _, a, _, _ in middles]
    # the middles' weights name the keys of this round: all of the aggregates' keys, or a
    # subset of them (a parameter-sharded round runs the keys of one wave at a time)
    keys = list(middles[0][0].keys())
    fusable = (all(isinstance(a, DeferredAggregate) and a._data is None and a._pending and _uniform(a)
                   for a in aggs)
               and len({len(a._pending) for a in aggs}) == 1
               and all(list(w.keys()) == keys and set(keys) <= set(a._keys) for w, a, _, _ in middles))
    device = None
    mid_stride = {}
    if fusable:
        device = engine.pick_device(middles[0][0])
        for k in keys:
            shape, dt = aggs[0]._meta[k]
            n = math.prod(shape)
            # middle weights: every middle contiguous, or every middle a tiled slot view of one
            # layout (an UpdateSlab holding the middles: a chunk's middles are one block)
            mw = [w[k] for w, _, _, _ in middles]
            st = mid_stride[k] = _tiled_stride(mw, n)
            if st is None or (st and any(t.dtype != dt or t.device != device for t in mw)):
                fusable = False
                break
            tensors = [] if st else mw
            if isinstance(top_agg, collections.abc.Mapping):
                tensors.append(top_agg[k])
            if top_weights is not None:
                tensors.append(top_weights[k] if k in top_weights else None)
            if (engine.dtype_code(dt) not in (engine.N.FLAME_F32, engine.N.FLAME_BF16, engine.N.FLAME_F16)
                    or any(t is None or t.dtype != dt or t.numel() != n or t.device != device
                           or not t.is_contiguous() for t in tensors)
                    or any(a._meta[k][1] != dt or math.prod(a._meta[k][0]) != n for a in aggs)):
                fusable = False
                break
    if fusable and update_middle_weights:
        # middles updated in place must not share tensors (the separate calls would chain them)
        fusable = all(len({w[k].data_ptr() for w, _, _, _ in middles}) == len(middles) for k in keys)
    if fusable:
        rows, keep = _hier_rows(aggs, keys, device)
        fusable = rows is not None
    if not fusable:
        res = _compose_hierarchy(middles, top_agg, version, top_weights, top_goal, with_delta,
                                 update_middle_weights)
        for gi in range(len(key_groups or ())):
            if after_group is not None:
                after_group(gi)
        return res

    top_accum = top_agg is not None
    if isinstance(top_agg, DeferredAggregate):
        top_agg.flush()
        top_out = top_agg._data
        result = top_agg
    elif top_agg is not None:
        top_out, result = top_agg, top_agg
    else:
        top_out = collections.OrderedDict(
            (k, torch.empty(aggs[0]._meta[k][0], dtype=aggs[0]._meta[k][1], device=device)) for k in keys)
        result = top_out
    deltas = None
    if with_delta:
        deltas = [{k: torch.empty(aggs[0]._meta[k][0], dtype=aggs[0]._meta[k][1], device=device) for k in keys}
                  for _ in middles]
    mid_rates = [[r for _, r in a._pending] for a in aggs]
    mid_goals = [g for _, _, g, _ in middles]
    for gi, g in enumerate(key_groups if key_groups is not None else [keys]):
        groups = collections.OrderedDict()
        for k in g:
            groups.setdefault(engine.dtype_code(aggs[0]._meta[k][1]), []).append(k)
        for code, ks in groups.items():
            segs = []
            for k in ks:
                ptrs, stride = rows[k]
                t_out = top_out[k]
                segs.append(engine.HierSeg(
                    numel=t_out.numel(), mid_w=[w[k].data_ptr() for w, _, _, _ in middles], clients=ptrs,
                    mid_delta=[d[k].data_ptr() for d in deltas] if deltas is not None else None,
                    top_w=top_weights[k].data_ptr() if top_weights is not None else 0,
                    top_in=t_out.data_ptr() if top_accum else 0, top_out=t_out.data_ptr(), tile_stride=stride,
                    mid_tile_stride=mid_stride[k]))
            engine.hier_fedbuff_(segs, code, mid_rates, mid_goals, top_rates, top_accum=top_accum,
                                 top_goal=top_goal if top_weights is not None else None, device=device, keep=keep,
                                 mid_readonly=not update_middle_weights)
        if after_group is not None:
            after_group(gi)
    engine._keepalive(keep, device)
    return result, deltas
