"""Parameter-sharded aggregation across the GPUs of a node.

Elements are independent and every reduction runs over clients per element, so
the model is cut by ELEMENTS, never by clients (a client split would need a
reduce-scatter and reorder the fp32 sum).  Each rank reduces only the elements it
owns -- with the same kernel and the same per-element client order, so the result
is bit-identical to one GPU and to the reference -- and an in-place RCCL
``all_gather_into_tensor`` over xGMI writes every rank's elements straight into
the model's own tensors (no pack / unpack pass on either side).

:class:`ShardPlan` decides ownership.  Per state_dict key of ``n`` elements, the
largest multiple of ``world * align`` (the key's *main* part) is split among the
ranks; the remainder (< ``world * align`` elements, the *tail*) is reduced by every
rank, so it needs no exchange.  The main parts of all keys, taken in model order,
are cut into a few *waves* of decreasing size (75 / 20 / 5 %); in a wave, each
*piece* ``[g0, g1)`` of a key is split into ``world`` equal contiguous ranges and
rank ``r`` owns the ``r``-th.  A wave is one kernel launch per dtype, and its
all-gather (in place: each rank's range already sits at its offset inside the
piece) starts as soon as the launch is queued, so it runs on the collective stream
while the next wave is reduced; only the last, smallest wave's exchange is exposed.

Each rank holds its slices of every client update -- ``DeviceUpdateCache(shard=plan)``
writes only the owned ranges of an arriving update into a tiled slab (a strided H2D
of those ranges) -- and the optimizer state that lives per element (FedOPT
``m_t`` / ``v_t`` / ``current_weights``, FedBuff aggregates, middle aggregators'
weights) exists only for the owned ranges and is never exchanged.

* :class:`ShardedOptimizer` -- any drop-in optimizer's ``do`` / ``scale_add_agg_weights``
  over a process group (configs 3/4 at N GPUs).
* :class:`ShardedHierarchy` -- a node's co-located two-level hierarchy (async FedBuff,
  ``asyncfl/middle_aggregator.py:164-256`` -> ``asyncfl/top_aggregator.py:54-115``, or
  synchronous FedAvg, ``syncfl/middle_aggregator.py:163-229`` ->
  ``syncfl/top_aggregator.py:122-176``) over a process group: config 5.

The wrapped optimizer / hierarchy function is whatever runs per rank: the HIP drop-ins
in the product; the CPU multi-process tests (gloo, world size 2) wrap the oracle.
"""
from __future__ import annotations

import collections
import math
import os
import weakref
from dataclasses import dataclass
from typing import Dict, Optional

import torch

from . import engine, shm_lease

ALIGN_ELEMS = 2048               # a multiple of every kernel chunk / slab tile (1024 fp32, 2048 bf16 / fp16)
DEFAULT_FRACS = (0.75, 0.20, 0.05)
# the hierarchy's workgroups are long (a chunk's 4096 arrivals): every extra launch costs a
# ramp-down tail, so it pipelines in two waves
HIER_FRACS = (0.9, 0.1)


@dataclass(frozen=True)
class Sub:
    """One local range of a key: a wave's piece ``[g0, g1)`` of which this rank owns
    ``[lo, hi)``, or the key's tail (``lo, hi == g0, g1``, reduced by every rank)."""
    name: str
    key: str
    wave: int
    g0: int
    g1: int
    lo: int
    hi: int
    tail: bool


class ShardPlan:
    """Which elements of every state_dict key this rank owns (see the module docstring).

    ``names`` are the local keys (``"<key>#<g0>"`` for a piece, ``"<key>#tail"``) in model
    order; a rank-local dict (of views, client slices, optimizer state) uses them.
    """

    def __init__(self, model, world: int, rank: int, *, align: int = ALIGN_ELEMS, fracs=DEFAULT_FRACS,
                 last_wave_quantum: int = 0):
        if not 0 <= rank < world:
            raise ValueError(f"rank {rank} outside world {world}")
        self.world, self.rank, self.align = int(world), int(rank), int(align)
        self.keys = list(model.keys())
        self.shapes = {k: tuple(engine.logical_shape(model, k)) for k in self.keys}
        self.dtypes = {k: engine.weight_dtype(model, k) for k in self.keys}
        self.numel = {k: math.prod(self.shapes[k]) for k in self.keys}
        unit = self.world * self.align
        main = {k: self.numel[k] // unit * unit for k in self.keys}
        total = sum(main.values())
        cuts, acc = [0], 0.0
        for f in fracs[:-1]:
            acc += f
            cuts.append(min(max(int(total * acc) // unit * unit, cuts[-1]), total))
        q = int(last_wave_quantum)
        if q > 0 and len(cuts) > 1 and q % self.align == 0 and total // self.world >= 2 * q:
            # the last wave's per-rank size -> the nearest whole multiple of q (>= 1): a launch
            # of long-lived workgroups then ends on a full round of them (ShardedHierarchy)
            n_q = max(1, round((total - cuts[-1]) / self.world / q))
            cuts[-1] = max(total - n_q * q * self.world, cuts[-2])
        cuts.append(total)
        subs, off = [], 0
        for k in self.keys:
            m = main[k]
            for w in range(len(cuts) - 1):
                a, b = max(cuts[w], off), min(cuts[w + 1], off + m)
                if a < b:
                    g0, g1 = a - off, b - off
                    per = (g1 - g0) // self.world
                    lo = g0 + self.rank * per
                    subs.append(Sub(f"{k}#{g0}", k, w, g0, g1, lo, lo + per, False))
            if m < self.numel[k] or self.numel[k] == 0:      # (an empty key keeps an empty tail)
                subs.append(Sub(f"{k}#tail", k, -1, m, self.numel[k], m, self.numel[k], True))
            off += m
        used = sorted({s.wave for s in subs if not s.tail})
        remap = {w: i for i, w in enumerate(used)}
        # tails ride the first wave (they need no exchange, so they never delay one)
        self.subs = [Sub(s.name, s.key, 0 if s.tail else remap[s.wave], s.g0, s.g1, s.lo, s.hi, s.tail)
                     for s in subs]
        self.by_name = {s.name: s for s in self.subs}
        self.names = [s.name for s in self.subs]
        self.n_waves = max(1, len(used))
        self.wave_names = [[s.name for s in self.subs if s.wave == w] for w in range(self.n_waves)]
        self.local_numel = {s.name: s.hi - s.lo for s in self.subs}
        self.local_shapes = {s.name: (s.hi - s.lo,) for s in self.subs}
        self.full_ranges = {s.name: (s.key, s.lo, s.hi) for s in self.subs}      # over a full-model slab
        self.self_ranges = {s.name: (s.name, 0, s.hi - s.lo) for s in self.subs}  # over a local slab
        self._restricted = {}
        self._local_slabs = weakref.WeakSet()

    # ---------------------------------------------------------------- layout
    def matches(self, model) -> bool:
        return (list(model.keys()) == self.keys
                and all(math.prod(engine.logical_shape(model, k)) == self.numel[k] for k in self.keys))

    def local_template(self) -> Dict[str, torch.Tensor]:
        """Shapes / dtypes of this rank's slices (an ``UpdateSlab`` template)."""
        return collections.OrderedDict((s.name, torch.empty(s.hi - s.lo, dtype=self.dtypes[s.key], device="meta"))
                                       for s in self.subs)

    def owned_elements(self) -> int:
        return sum(s.hi - s.lo for s in self.subs)

    def views(self, flat: Dict[str, torch.Tensor], names=None):
        """``{name: flat[key][lo:hi]}`` -- in-place views of 1-D model tensors."""
        by = self.by_name
        return collections.OrderedDict((n, flat[by[n].key][by[n].lo:by[n].hi]) for n in (names or self.names))

    # ---------------------------------------------------------------- client updates
    def slice_update(self, weights):
        """This rank's slices of a full client update as plain views / host slices (what
        ``DeviceUpdateCache(shard=plan)`` copies to the device)."""
        for k, t in weights.items():
            if k not in self.numel:
                raise KeyError(k)
            if isinstance(t, torch.Tensor) and not t.is_cuda:
                shm_lease.check_live(t)     # the slices below no longer carry the segment's stamp
        out = collections.OrderedDict()
        for s in self.subs:
            if s.key in weights:
                out[s.name] = _slice(weights[s.key], s.lo, s.hi, self.numel[s.key])
        return out

    def _is_local_slab(self, slab) -> bool:
        if slab in self._local_slabs:
            return True
        ok = (slab.keys == self.names
              and all(slab.meta[n][0] == self.dtypes[self.by_name[n].key] and slab.meta[n][2] == self.local_numel[n]
                      for n in self.names))
        if ok:
            self._local_slabs.add(slab)
        return ok

    def local(self, weights):
        """A client update as this rank sees it: local names -> its slices.

        * a slot of a slab that already holds only this rank's slices: unchanged;
        * a slot of a full-model slab: a :class:`~flame_amd.slab.SlabRef` (no views made;
          the engine computes pointer rows from slot numbers);
        * a dict already keyed by this plan's local names: unchanged;
        * a dict of tensors (device, pinned or pageable host): views / slices.
        """
        slab = getattr(weights, "slab", None)
        rng = getattr(weights, "ranges", None)
        if slab is not None and (rng is self.full_ranges or rng is self.self_ranges):
            return weights                      # already this plan's slices (a SlabRef it made)
        if slab is not None and rng is None:
            if self._is_local_slab(slab):
                return weights
            if all(s.key in slab.meta and slab.meta[s.key][0] == self.dtypes[s.key]
                   and slab.meta[s.key][2] == self.numel[s.key]
                   and s.lo % slab.storage[self.dtypes[s.key]].shape[2] == 0 for s in self.subs):
                from .slab import SlabRef
                return SlabRef(slab, weights.slot, self.full_ranges, self.local_shapes, owner=weights)
        if slab is None and weights and all(k in self.by_name and k not in self.numel for k in weights.keys()):
            return weights     # already this rank's slices, one tensor per range (DeviceUpdateCache(shard=plan)
                               # keeps a model it cannot slab -- bool / uint8 buffers -- that way)
        return self.slice_update(weights)

    def restrict(self, weights, wave: int):
        """A local client update restricted to one wave's names."""
        names = self.wave_names[wave]
        slab = getattr(weights, "slab", None)
        if slab is not None:
            from .slab import SlabRef
            ranges = getattr(weights, "ranges", None)
            if ranges is None and self._is_local_slab(slab):
                ranges = self.self_ranges
            if ranges is self.self_ranges or ranges is self.full_ranges:
                key = (id(ranges), wave)
                table = self._restricted.get(key)
                if table is None:
                    table = self._restricted[key] = {n: ranges[n] for n in names}
                return SlabRef(slab, weights.slot, table, self.local_shapes, owner=getattr(weights, "_owner", None)
                               or weights)
        return {n: weights[n] for n in names if n in weights}


def _slice(t: torch.Tensor, lo: int, hi: int, numel: int) -> torch.Tensor:
    """Elements [lo, hi) of a tensor of ``numel`` logical elements (tiled slab views stay tiled
    when ``lo`` starts a tile)."""
    if t.is_cuda and engine.tiled_stride(t, numel) and lo % t.shape[1] == 0:
        return engine.slice_elems(t, lo, hi, numel)
    return t.reshape(-1)[:numel][lo:hi]


# -------------------------------------------------------------------- collectives
# one coalesced group per wave (RCCL: a single grouped launch); False = one async collective
# per piece through the public API only (FLAME_AMD_COALESCE=0)
COALESCE = os.environ.get("FLAME_AMD_COALESCE", "1") != "0"
# collectives issued per path ("coalesced" groups, "async" single gathers, "host_staged"), for tests
GATHER_STATS = collections.Counter()
# None, or a list that every call's in-place gathers are timed into (bench.py's N > 1 lines):
# (wave, bytes this rank received, start, end) with start marked on the launch stream right before
# the wave's collective is issued (behind the wave's kernels) and end right after its work.wait()
# -- CUDA events for device tensors, host perf_counter seconds for CPU tensors.  A wave's span is
# its gather's time plus whatever later kernels the launch stream ran before the wait: exact for
# the last wave, an upper bound for the hidden ones.
GATHER_TIMING = None


def _mark_like(start):
    """A mark of the same kind as ``start`` (a CUDA event on the current stream, or a host time)."""
    if isinstance(start, float):
        import time
        return time.perf_counter()
    ev = torch.cuda.Event(enable_timing=True)
    ev.record()
    return ev


def _mark(t: torch.Tensor):
    if t.is_cuda:
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(torch.cuda.current_stream(t.device))
        return ev
    import time
    return time.perf_counter()


def _coalescing_manager():
    """torch's private ``_coalescing_manager`` context factory, or None if this torch lacks it."""
    try:
        from torch.distributed.distributed_c10d import _coalescing_manager as cm
    except ImportError:
        return None
    return cm


class _Comm:
    """The process group (none at world 1) and the in-place all-gathers of one call."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.group = group
        self.dist = dist if (dist.is_available() and dist.is_initialized()) else None
        self.world = dist.get_world_size(group) if self.dist else 1
        self.rank = dist.get_rank(group) if self.dist else 0
        self.backend = dist.get_backend(group) if self.dist else None
        self.coalesce = COALESCE
        self._works = []
        self._timing = []       # (wave, bytes received, start mark) of gathers issued since the last wait

    def _fail(self, wave, what, e):
        raise RuntimeError(f"flame_amd.shard: rank {self.rank} of {self.world} ({self.backend}): {what} of "
                           f"wave {wave} failed: {e}") from e

    def all_gather_inplace(self, pairs, wave=None) -> None:
        """``pairs``: [(piece, owned)] with ``owned`` this rank's range inside ``piece``.
        A failing collective raises naming this rank and ``wave``.

        One body for RCCL and for gloo on CPU tensors (the world 2 / 3 / 8 CPU tests run it):
        async, in place (NCCL's in-place all-gather, ``sendbuff == recvbuff + rank * count``),
        the call's pieces of one dtype in one coalesced group (``_coalescing_manager``; without it -- a torch
        that lacks the private helper, or ``coalesce=False`` -- one async public
        ``all_gather_into_tensor`` per piece).  Only gloo with CUDA tensors (tests where ranks
        share one GPU; gloo has no device all-gather) stages through the host synchronously."""
        if not pairs or self.dist is None:
            return
        if GATHER_TIMING is not None:
            recv = sum((p.numel() - o.numel()) * p.element_size() for p, o in pairs)
            self._timing.append((wave, recv, _mark(pairs[0][0])))
        try:
            self._all_gather_inplace(pairs, wave)
        except Exception as e:  # noqa: BLE001 - re-raised with the rank and wave
            self._fail(wave, "all-gather", e)

    def _all_gather_inplace(self, pairs, wave) -> None:
        d = self.dist
        if self.backend == "gloo" and pairs[0][0].is_cuda:
            for piece, owned in pairs:
                host = torch.empty(piece.numel(), dtype=piece.dtype)
                d.all_gather_into_tensor(host, owned.cpu(), group=self.group)
                piece.copy_(host)
            GATHER_STATS["host_staged"] += len(pairs)
            return
        cm_factory = _coalescing_manager() if self.coalesce else None
        by_dtype = collections.OrderedDict()
        for piece, owned in pairs:
            by_dtype.setdefault(piece.dtype, []).append((piece, owned))
        for group in by_dtype.values():
            # one group per dtype: gloo's coalesced all-gather flattens a group into ONE buffer of
            # its first tensor's dtype (a bf16 + fp32 group came back with the fp32 values rounded
            # to bf16); RCCL would take mixed dtypes, the per-dtype split costs it nothing measurable
            if cm_factory is None or len(group) == 1:
                for piece, owned in group:
                    self._works.append((wave, d.all_gather_into_tensor(piece, owned, group=self.group,
                                                                       async_op=True)))
                GATHER_STATS["async"] += len(group)
                continue
            with cm_factory(group=self.group, async_ops=True) as cm:
                for piece, owned in group:
                    d.all_gather_into_tensor(piece, owned, group=self.group)
            self._works.append((wave, cm))
            GATHER_STATS["coalesced"] += 1

    def wait(self) -> None:
        """Order the launch stream after every gather issued so far (host does not block)."""
        works, self._works = self._works, []
        timing, self._timing = self._timing, []
        starts = {wave: (recv, start) for wave, recv, start in timing}
        for i, (wave, w) in enumerate(works):
            try:
                w.wait()
            except Exception as e:  # noqa: BLE001 - re-raised with the rank and wave
                self._fail(wave, "wait on the all-gather", e)
            if wave in starts and (i + 1 == len(works) or works[i + 1][0] != wave):
                # right after the wave's last wait: the launch stream reaches this mark once the
                # kernels queued so far and gathers 0..wave are done
                self._timed(wave, *starts.pop(wave))
        for wave, (recv, start) in starts.items():      # host-staged gathers: done at issue
            self._timed(wave, recv, start)

    @staticmethod
    def _timed(wave, recv, start) -> None:
        if GATHER_TIMING is not None:
            GATHER_TIMING.append((wave, recv, start, _mark_like(start)))


class _Work:
    """The model's tensors as flat vectors on ``device`` that kernels and collectives write
    in place; a tensor that is not contiguous there is staged and written back."""

    def __init__(self, weights, keys, device):
        self.flat, self._staged = {}, []
        for k in keys:
            t = weights[k]
            if t.device == device and t.is_contiguous():
                self.flat[k] = t.view(-1)
            else:
                d = torch.empty(t.numel(), dtype=t.dtype, device=device)
                d.copy_(t.reshape(-1))
                self.flat[k] = d
                self._staged.append((t, d))

    def writeback(self) -> None:
        for t, d in self._staged:
            t.copy_(d.view(t.shape))


class _Gatherer:
    """Routes each local result into the full tensor it belongs to (the model's own when the
    wrapped call wrote in place, else a new tensor of the result's dtype) and all-gathers
    wave by wave."""

    def __init__(self, comm: _Comm, plan: ShardPlan, weights, work: _Work):
        self.comm, self.plan, self.weights, self.work = comm, plan, weights, work
        self.target = {}
        self.new = collections.OrderedDict()
        self.inplace = collections.defaultdict(list)
        self.issued = set()

    def expect_inplace(self) -> None:
        """The wrapped call writes every local name in place (before it starts issuing)."""
        for s in self.plan.subs:
            self.target[s.name] = self.work.flat[s.key]
            self.inplace[s.key].append(s)

    def check_inplace(self, res, local) -> None:
        for n in self.plan.names:
            r, v = res[n], local[n]
            if not (r is v or (r.dtype == v.dtype and r.numel() == v.numel() and r.data_ptr() == v.data_ptr())):
                raise RuntimeError(f"flame_amd.shard: {n} was expected in place")

    def collect(self, res, local, names) -> None:
        by = self.plan.by_name
        for n in names:
            s = by[n]
            r, v = res[n], local[n]
            if r is v or (r.device == v.device and r.dtype == v.dtype and r.numel() == v.numel()
                          and r.data_ptr() == v.data_ptr()):
                self.target[n] = self.work.flat[s.key]
                self.inplace[s.key].append(s)
                continue
            t = self.new.get(s.key)
            if t is None:
                t = self.new[s.key] = torch.empty(self.plan.numel[s.key], dtype=r.dtype, device=v.device)
            t[s.lo:s.hi].copy_(r.reshape(-1))
            self.target[n] = t

    def alloc(self, name, dtype, shape) -> torch.Tensor:
        """Where a wrapped optimizer writes local result ``name``: its range of a new full
        tensor of ``dtype`` (gathered in place when the name's wave is issued)."""
        s = self.plan.by_name[name]
        t = self.new.get(s.key)
        if t is None or t.dtype != dtype:
            t = self.new[s.key] = torch.empty(self.plan.numel[s.key], dtype=dtype,
                                              device=self.work.flat[s.key].device)
        self.target[name] = t
        return t[s.lo:s.hi].view(shape)

    def issue(self, wave: int) -> None:
        if wave in self.issued:
            return
        self.issued.add(wave)
        by = self.plan.by_name
        pairs = []
        for n in self.plan.wave_names[wave]:
            s = by[n]
            if not s.tail and n in self.target:
                t = self.target[n]
                pairs.append((t[s.g0:s.g1], t[s.lo:s.hi]))
        self.comm.all_gather_inplace(pairs, wave)

    def finish(self):
        """Issue what is left, wait for the gathers; the caller's dict (in place) or a new
        dict with new tensors."""
        for w in range(self.plan.n_waves):
            self.issue(w)
        self.comm.wait()
        self.work.writeback()
        if not self.new:
            return self.weights
        for k, subs in self.inplace.items():      # a key partly in place: its gathered ranges join
            if k in self.new:
                for s in subs:
                    self.new[k][s.g0:s.g1].copy_(self.work.flat[k][s.g0:s.g1])
        return collections.OrderedDict(
            (k, self.new[k].view(self.plan.shapes[k]) if k in self.new else self.weights[k]) for k in self.plan.keys)


# -------------------------------------------------------------------- cache adapters
class _SlicedResult:
    """TrainResult-shaped record carrying this rank's slices of a client's weights."""

    __slots__ = ("weights", "count", "version")

    def __init__(self, weights, count, version):
        self.weights, self.count, self.version = weights, count, version


class _SliceCache:
    """A view of the caller's cache that hands out this rank's slices of every entry, in the
    caller's ``iterkeys()`` order; popping it pops the caller's entry."""

    def __init__(self, cache, plan: ShardPlan):
        self._cache, self._plan = cache, plan

    def __len__(self):
        return len(self._cache)

    def iterkeys(self):
        return self._cache.iterkeys()

    def pop(self, key, default=None):
        tres = self._cache.pop(key, default)
        if tres is None or tres is default:
            return tres
        lw = self._plan.local(tres.weights)
        if lw is tres.weights:          # already this rank's slices (rank-local slab slot)
            return tres
        return _SlicedResult(lw, getattr(tres, "count", 0), getattr(tres, "version", 0))


class _Replay:
    """Records drained from the caller's cache once, replayed in the same order (one replay
    per wave)."""

    def __init__(self, items):
        self._d = collections.OrderedDict(items)

    def __len__(self):
        return len(self._d)

    def __contains__(self, key):
        return key in self._d

    def __getitem__(self, key):
        return self._d[key]

    def iterkeys(self):
        return iter(list(self._d))

    def pop(self, key, default=None):
        return self._d.pop(key, default)


def _drain(cache, plan: ShardPlan):
    """``cache.pop`` in ``cache.iterkeys()`` order (fedavg.py:79-82), each record sliced; a
    record already holding this rank's slices (a slot of the rank-local slab) is kept as is."""
    out = []
    local_slab = None
    for k in list(cache.iterkeys()):
        tres = cache.pop(k)
        if tres is None:
            continue
        w = tres.weights
        slab = getattr(w, "slab", None)
        if slab is not None and slab is local_slab and getattr(w, "ranges", None) is None:
            out.append((k, tres))
            continue
        lw = plan.local(w)
        if lw is w:
            if slab is not None and getattr(w, "ranges", None) is None:
                local_slab = slab
            out.append((k, tres))
        else:
            out.append((k, _SlicedResult(lw, getattr(tres, "count", 0), getattr(tres, "version", 0))))
    return out


def _restrict(plan: ShardPlan, rec, wave: int) -> _SlicedResult:
    return _SlicedResult(plan.restrict(rec.weights, wave), getattr(rec, "count", 0), getattr(rec, "version", 0))


def _fedopt_round(inner) -> bool:
    """flame_amd's FedOPT with state: its next round is a fused adaptive step."""
    from .optimizer.fedopt import FedOPT
    return isinstance(inner, FedOPT) and inner.current_weights is not None


def _device_of(weights, device):
    if device is not None:
        return torch.device(device)
    for t in weights.values():
        if isinstance(t, torch.Tensor) and t.is_cuda:
            return t.device
    if torch.cuda.is_available():
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def _stateless(inner) -> bool:
    """``do`` keeps no state between calls, so it may run wave by wave."""
    from .optimizer.fedavg import FedAvg
    from .optimizer.fedprox import FedProx
    return type(inner) in (FedAvg, FedProx)


# -------------------------------------------------------------------- optimizers
class ShardedOptimizer:
    """Any flame optimizer's ``do()`` executed parameter-sharded over a process group.

    Every rank calls ``do`` with the same ``base_weights`` (the full model) and a cache of
    the same client updates -- whole updates (sliced here: views, or slab-slot references)
    or, normally, only this rank's slices (``DeviceUpdateCache(shard=opt.plan)``).  Each
    rank runs the wrapped optimizer on its slices; the results are gathered in place.

    * FedAvg / FedProx (stateless ``do``): one wrapped ``do`` per wave on the cache's
      records replayed, each wave's all-gather overlapping the next wave's reduction;
      ``base_weights`` is mutated in place and returned (fedavg.py:74,87).
    * FedOPT and other stateful optimizers: one wrapped ``do`` over all local names, then
      the gathers.  A result written in place lands in ``base_weights``; new result tensors
      (FedOPT's ``current_weights``, fedopt.py:125-129, incl. integer buffers it promotes)
      are gathered into NEW full tensors, returned in a new dict, as the reference does.
      The state (``m_t``, ``v_t``, ``current_weights``, ``agg_weights``) stays sharded: only
      the owned ranges of ``base_weights`` receive the average.  An empty round returns
      the previous round's gathered dict (the reference returns ``current_weights``).
    * FedBuff (``accumulate_only=True``): ``do`` returns the wrapped optimizer's aggregate
      of this rank's slices (it stays sharded); ``scale_add_agg_weights(base_weights, agg,
      goal)`` applies it on the owned ranges and gathers.  Call ``set_layout(model)`` first.

    Per element the arithmetic is the wrapped optimizer's, so results are bit-identical to
    one process.
    """

    ALIGN_ELEMS = ALIGN_ELEMS

    def __init__(self, inner, group=None, device: Optional[torch.device] = None, accumulate_only: bool = False,
                 *, waves: Optional[bool] = None, fracs=DEFAULT_FRACS, align: int = ALIGN_ELEMS,
                 plan: Optional[ShardPlan] = None, gather: bool = True):
        self.inner = inner
        # gather=False (FedAvg / FedProx): no all-gathers -- each rank's base_weights is current on its
        # owned ranges (and the replicated tails) only, one launch over them; for a caller whose next
        # use of the model is host-side, e.g. flame_amd.egress.ShardedEgress writing every rank's
        # ranges straight into one host payload over each rank's own PCIe link
        self.gather = gather
        self.comm = _Comm(group)
        self.device = device
        self.accumulate_only = accumulate_only
        self.waves = waves
        self.fracs, self.align = fracs, align
        self.plan = plan
        self._last_local = self._last_full = None

    @property
    def world(self):
        return self.comm.world

    @property
    def rank(self):
        return self.comm.rank

    def set_layout(self, model_weights) -> None:
        """The model whose keys are sharded (FedBuff: the role's self.weights)."""
        self.plan = ShardPlan(model_weights, self.world, self.rank, align=self.align, fracs=self.fracs)

    def _ensure_plan(self, weights) -> ShardPlan:
        if self.plan is None or not self.plan.matches(weights):
            self.set_layout(weights)
        return self.plan

    def _gather_all(self, res, local, gat: _Gatherer):
        gat.collect(res, local, [n for n in self.plan.names if n in res])
        for w in range(self.plan.n_waves):
            gat.issue(w)
        return gat.finish()

    # ---------------------------------------------------------------- optimizer contract
    def do(self, base_weights, cache, *, total: int = 0, version: int = 0, **kwargs):
        if self.accumulate_only:
            return self._accumulate(base_weights, cache, total, version, kwargs)
        assert base_weights is not None
        plan = self._ensure_plan(base_weights)
        work = _Work(base_weights, plan.keys, _device_of(base_weights, self.device))
        local = plan.views(work.flat)
        gat = _Gatherer(self.comm, plan, base_weights, work)
        if len(cache) == 0 or total == 0:
            res = self.inner.do(local, cache, total=total, version=version, **kwargs)
            if res is None:
                return None
            if res is self._last_local:
                return self._last_full
            return self._remember(res, self._gather_all(res, local, gat))
        records = _drain(cache, plan)
        if not self.gather:
            # one do() over all local names (no waves: they exist to overlap the gathers); the
            # wrapped optimizer must write in place, as FedAvg / FedProx do (fedavg.py:74,87)
            res = self.inner.do(local, _Replay(records), total=total, version=version, **kwargs)
            if res is None:
                return None
            try:
                gat.check_inplace(res, local)
            except RuntimeError as e:
                raise NotImplementedError(f"ShardedOptimizer(gather=False) needs an in-place optimizer "
                                          f"(FedAvg / FedProx): {e}") from e
            work.writeback()
            return base_weights
        if _stateless(self.inner) and self.waves is not False:
            # flame_amd FedAvg / FedProx: one do(), one launch per wave (pointer rows built once),
            # each wave's in-place all-gather queued right behind its launch
            gat.expect_inplace()
            res = self.inner.do(local, _Replay(records), total=total, version=version,
                                flame_amd_key_groups=plan.wave_names, flame_amd_after_group=gat.issue, **kwargs)
            if res is None:
                return None
            gat.check_inplace(res, local)
            return gat.finish()
        if _fedopt_round(self.inner) and self.waves is not False:
            # flame_amd FedOPT past its passthrough round: one do(), one launch per wave writing
            # the new `current` straight into the full tensors, each wave gathered right behind
            res = self.inner.do(local, _Replay(records), total=total, version=version,
                                flame_amd_key_groups=plan.wave_names, flame_amd_after_group=gat.issue,
                                flame_amd_out_alloc=gat.alloc, **kwargs)
            if res is None:
                return None
            missing = [n for n in plan.names if n in res and n not in gat.target]
            if missing:      # not produced through the allocator: gathered after the fact
                gat.collect(res, local, missing)
                # re-issue only the waves holding such names (the others went out behind their launches)
                gat.issued -= {plan.by_name[n].wave for n in missing}
            return self._remember(res, gat.finish())
        if self.waves:
            # any other stateless optimizer (e.g. the CPU oracle in tests): one do() per wave on
            # the records replayed, each wave gathered as soon as it is done
            for w in range(plan.n_waves):
                names = plan.wave_names[w]
                lb = collections.OrderedDict((n, local[n]) for n in names)
                res = self.inner.do(lb, _Replay([(k, _restrict(plan, r, w)) for k, r in records]), total=total,
                                    version=version, **kwargs)
                if res is None:
                    return None
                gat.collect(res, lb, names)
                gat.issue(w)
            return gat.finish()
        res = self.inner.do(local, _Replay(records), total=total, version=version, **kwargs)
        if res is None:
            return None
        return self._remember(res, self._gather_all(res, local, gat))

    def _remember(self, local_res, full):
        self._last_local, self._last_full = local_res, full
        return full

    def _accumulate(self, agg, cache, total, version, kwargs):
        if len(cache) == 0 or total == 0:
            return self.inner.do(agg, cache, total=total, version=version, **kwargs)
        if self.plan is None:
            raise RuntimeError("ShardedOptimizer(accumulate_only): call set_layout(model_weights) first")
        return self.inner.do(agg, _SliceCache(cache, self.plan), total=total, version=version, **kwargs)

    def do_arrivals(self, agg, arrivals, *, version: int = 0):
        """FedBuff's batched arrivals (``FedBuff.do_arrivals``) on this rank's slices of each
        arrival (``accumulate_only``); the aggregate stays sharded."""
        if not self.accumulate_only:
            raise TypeError("ShardedOptimizer.do_arrivals: FedBuff with accumulate_only=True only")
        if self.plan is None:
            raise RuntimeError("ShardedOptimizer(accumulate_only): call set_layout(model_weights) first")
        plan, local = self.plan, []
        local_slab = None         # a slab already known to hold only this rank's slices
        for tres in arrivals:
            w = tres.weights
            slab = getattr(w, "slab", None)
            if slab is not None and slab is local_slab and getattr(w, "ranges", None) is None:
                local.append(tres)
                continue
            lw = plan.local(w)
            if lw is w and slab is not None and getattr(w, "ranges", None) is None:
                local_slab = slab
            local.append(tres if lw is w else _SlicedResult(lw, getattr(tres, "count", 0), getattr(tres, "version", 0)))
        return self.inner.do_arrivals(agg, local, version=version)

    def scale_add_agg_weights(self, base_weights, agg_goal_weights, agg_goal: int):
        """fedbuff.py:101-127 on this rank's ranges of ``base_weights``, then the in-place gather."""
        plan = self._ensure_plan(base_weights)
        work = _Work(base_weights, plan.keys, _device_of(base_weights, self.device))
        local = plan.views(work.flat)
        gat = _Gatherer(self.comm, plan, base_weights, work)
        from .optimizer.fedbuff import FedBuff
        if isinstance(self.inner, FedBuff):
            # flame_amd FedBuff: one launch per wave in place, each wave's gather right behind it
            gat.expect_inplace()
            res = self.inner.scale_add_agg_weights(local, agg_goal_weights, agg_goal,
                                                   flame_amd_key_groups=plan.wave_names,
                                                   flame_amd_after_group=gat.issue)
            gat.check_inplace(res, local)
            return gat.finish()
        res = self.inner.scale_add_agg_weights(local, agg_goal_weights, agg_goal)
        return self._gather_all(res, local, gat)

    def __getattr__(self, name):              # regularizer, m_t, v_t, ... of the wrapped optimizer
        inner = self.__dict__.get("inner")
        if inner is None:
            raise AttributeError(name)
        return getattr(inner, name)


# -------------------------------------------------------------------- config 5
def _hier_wave_quantum(model, device, middles: int, sync: bool) -> int:
    """Per-rank elements of one full round of resident hierarchy workgroups on ``device``
    (for the dtype of the model's largest key), a multiple of ALIGN_ELEMS; 0 if unknown."""
    if device is None or torch.device(device).type != "cuda" or not model:
        return 0
    big = max(model.keys(), key=lambda k: math.prod(engine.logical_shape(model, k)))
    code = engine.DTYPE_CODE.get(engine.weight_dtype(model, big))
    if code not in (engine.N.FLAME_F32, engine.N.FLAME_BF16, engine.N.FLAME_F16):
        return 0
    per_cu = engine.hier_resident_per_cu(code, int(middles), sync)
    cus = torch.cuda.get_device_properties(torch.device(device)).multi_processor_count
    q = per_cu * cus * engine.chunk_elems(code)
    return q if q % ALIGN_ELEMS == 0 else 0


class ShardedHierarchy:
    """A node's co-located two-level hierarchy, parameter-sharded over the node's GPUs
    (BASELINE.json config 5: hierarchical FedBuff, 4096 clients x 125M bf16 over 8 MI355X).

    Every rank holds its slices of every arrival (``DeviceUpdateCache(shard=hier.plan)``),
    of every middle aggregator's weights and FedBuff aggregate, and of the top's aggregate;
    per wave it runs the one-pass hierarchy (``hierarchy_round`` / ``sync_hierarchy_round``,
    one ``flame_hier_fedbuff`` launch per dtype) on the wave's names and all-gathers the top
    model's pieces in place -- the only data that crosses GPUs.  Bit-identical to running
    the whole hierarchy in one process (same per-element op sequence).

    * ``middle_optimizer()``: the middles' FedBuff (``asyncfl/middle_aggregator.py:164-203``,
      one arrival per ``do``) on this rank's slices.
    * ``round(middles, top_agg, version=, top_weights=, top_goal=)``: each middle's
      ``scale_add`` + upload delta (``:221-226,246``), the top's FedBuff over the deltas
      (``asyncfl/top_aggregator.py:85-92``) and its ``scale_add`` (``:103-110``).
    * ``sync_round(middles, top_weights)``: the synchronous hierarchy.

    ``middles`` (the node's fan-out, if known up front) sizes the last wave to a whole
    round of the hierarchy kernel's resident workgroups on ``device`` (a workgroup lives
    for all of a chunk's arrivals, so a launch ending on a partial round idles most of the
    GPU for one workgroup lifetime); ``sync`` says which kernel mode the rounds will use.
    """

    def __init__(self, model, group=None, device: Optional[torch.device] = None, *, fracs=HIER_FRACS,
                 align: int = ALIGN_ELEMS, round_fn=None, sync_round_fn=None, middles: Optional[int] = None,
                 sync: bool = False):
        self.comm = _Comm(group)
        q = _hier_wave_quantum(model, device, middles, sync) if middles else 0
        self.plan = ShardPlan(model, self.comm.world, self.comm.rank, align=align, fracs=fracs,
                              last_wave_quantum=q)
        self.device = device
        self._round_fn, self._sync_fn = round_fn, sync_round_fn

    def middle_optimizer(self, inner=None) -> ShardedOptimizer:
        if inner is None:
            from .optimizer.fedbuff import FedBuff
            inner = FedBuff()
        return ShardedOptimizer(inner, self.comm.group, self.device, accumulate_only=True, plan=self.plan)

    def local_model(self, weights):
        """This rank's ranges of a full model dict as in-place views (a dict keyed by the
        plan's local names -- sharded middle weights -- passes through)."""
        if list(weights.keys()) == self.plan.names:
            return weights
        out = collections.OrderedDict()
        for s in self.plan.subs:
            t = weights[s.key]
            if not t.is_contiguous():
                raise ValueError(f"ShardedHierarchy: {s.key} must be contiguous (updated in place)")
            out[s.name] = t.view(-1)[s.lo:s.hi]
        return out

    def _top(self, top_weights):
        if top_weights is None:
            return None, None, None
        work = _Work(top_weights, self.plan.keys, _device_of(top_weights, self.device))
        return self.plan.views(work.flat), work, _Gatherer(self.comm, self.plan, top_weights, work)

    def round(self, middles, top_agg=None, *, version: int, top_weights=None, top_goal=None,
              with_delta: bool = False, update_middle_weights: bool = True):
        """``middles``: ``(mid_weights, mid_agg, mid_goal, mid_version)`` as for
        ``hierarchy_round``; ``mid_agg`` from ``middle_optimizer().do``.  Returns
        ``(top_agg, deltas)`` -- both sharded (local names); ``top_weights`` (full model) is
        updated in place on every rank."""
        if self._round_fn is None:
            from .optimizer.fedbuff import hierarchy_round
            self._round_fn = hierarchy_round
        plan = self.plan
        mids = [(self.local_model(w), a, g, mv) for w, a, g, mv in middles]
        top_local, _, gat = self._top(top_weights)
        data = None
        if top_agg is not None:
            data = top_agg.materialize() if hasattr(top_agg, "materialize") else top_agg
            data = collections.OrderedDict((n, data[n]) for n in plan.names)
        if gat is not None:
            gat.expect_inplace()
        res, deltas = self._round_fn(mids, data, version=version, top_weights=top_local, top_goal=top_goal,
                                     with_delta=with_delta, update_middle_weights=update_middle_weights,
                                     key_groups=plan.wave_names, after_group=gat.issue if gat is not None else None)
        if gat is not None:
            gat.finish()
        return (top_agg if top_agg is not None else res), deltas

    def sync_round(self, middles, top_weights, *, with_delta: bool = False, update_middle_weights: bool = True):
        """``middles``: ``(mid_weights, cache, total)`` as for ``sync_hierarchy_round``; every
        cache is drained once (FedAvg.do's order) and replayed per wave.  Returns
        ``(top_weights, deltas)``; ``top_weights`` updated in place on every rank."""
        if self._sync_fn is None:
            from .optimizer.sync_hierarchy import sync_hierarchy_round
            self._sync_fn = sync_hierarchy_round
        plan = self.plan
        specs = []
        for w, cache, total in middles:
            if len(cache) == 0 or total == 0:
                raise ValueError("sync_round: every middle needs >= 1 update and total > 0")
            specs.append((self.local_model(w), _Replay(_drain(cache, plan)), total))
        top_local, _, gat = self._top(top_weights)
        gat.expect_inplace()
        _, deltas = self._sync_fn(specs, top_local, with_delta=with_delta, update_middle_weights=update_middle_weights,
                                  key_groups=plan.wave_names, after_group=gat.issue)
        gat.finish()
        return top_weights, deltas


__all__ = ["ShardPlan", "ShardedOptimizer", "ShardedHierarchy", "ALIGN_ELEMS", "DEFAULT_FRACS"]


def plan_for(model, group=None, **kw) -> ShardPlan:
    """The plan a ShardedOptimizer over ``group`` (default ``fracs`` / ``align``) would use for
    ``model`` (e.g. for ``DeviceUpdateCache(shard=...)`` before the optimizer has seen a model).
    Not a ShardedHierarchy's plan (other wave fractions, a last wave sized by the kernel's
    residency): use ``hier.plan`` there."""
    c = _Comm(group)
    return ShardPlan(model, c.world, c.rank, **kw)

