"""A node's co-located synchronous two-level hierarchy in one pass.

In flame's synchronous hierarchy every middle aggregator runs FedAvg over its
trainers (mode/horizontal/syncfl/middle_aggregator.py:163-204:
``self.weights = optimizer.do(deepcopy(self.weights), cache, total=total)``), then
uploads ``delta = weights - prev_weights`` with its sample count
(:206-229, common/util.py:152-159); the top aggregator runs FedAvg over the
middles' deltas (syncfl/top_aggregator.py:122-176, rate ``count/total``).  The
LIFL coordinated leaf aggregator uploads the same delta
(lifl_coord_syncfl/leaf_aggregator.py:155-173).

When the middles of one node share a GPU, ``sync_hierarchy_round`` runs the
whole round as ONE ``flame_hier_fedbuff`` launch per dtype with
``FLAME_HIER_SYNC``: per chunk, every middle's FedAvg is reduced in registers,
its new weights stored, its delta formed and added straight into the top's
FedAvg -- the deltas never touch HBM unless asked for.  Every op rounds as the
reference's torch-CPU sequence does, so the results are bit-identical to the
separate ``FedAvg.do`` / delta / ``FedAvg.do`` calls (the fallback, used for keys
the kernel does not take: integer buffers, mixed dtypes, ragged layouts).
"""
import collections

import numpy as np
import torch

from .. import _native as N
from .. import elementwise as ew, engine
from .fedbuff import _tiled_stride, _write_tiled

_KERNEL_DTYPES = (N.FLAME_F32, N.FLAME_BF16, N.FLAME_F16)


def _drain(cache, total):
    """FedAvg.do's draining (fedavg.py:79-84): (weights, count/total) in cache.iterkeys() order."""
    entries = []
    for k in list(cache.iterkeys()):
        tres = cache.pop(k)
        entries.append((tres.weights, tres.count / total))
    return entries


def sync_hierarchy_round(middles, top_weights, *, with_delta: bool = False, update_middle_weights: bool = True,
                         key_groups=None, after_group=None):
    """One synchronous round of a node's co-located hierarchy.

    ``middles``: ``(mid_weights, cache, total)`` per middle, in the order the top's
    cache yields their uploads (its ``cache.iterkeys()``); each ``cache`` is drained as
    ``FedAvg.do`` drains it.  ``top_weights`` is the top's model: it receives the
    top's FedAvg of the middles' deltas (rate ``total_m / Σ total``) in place.  Middle
    weights are updated in place (``update_middle_weights=False`` leaves them alone:
    only their deltas feed the top).  Returns ``(top_weights, deltas or None)``.

    Every middle needs at least one update and ``total > 0`` (a middle whose FedAvg
    returns None uploads nothing new in the reference; leave it out of ``middles``).

    ``key_groups`` / ``after_group``: one launch per dtype per group of keys, in order,
    ``after_group(i)`` called once group ``i`` is final (as for ``engine.accumulate``).
    """
    middles = list(middles)
    if not middles:
        raise ValueError("sync_hierarchy_round: no middles")
    totals = []
    entries = []
    for w, cache, total in middles:
        if len(cache) == 0 or total == 0:
            raise ValueError("sync_hierarchy_round: every middle needs >= 1 update and total > 0")
        totals.append(total)
        entries.append(_drain(cache, total))
    top_total = sum(totals)
    top_rates = [t / top_total for t in totals]
    mids = [w for w, _, _ in middles]
    keys = list(top_weights.keys())
    device = engine.pick_device(top_weights, *mids)

    fused = _fusable_keys(keys, mids, entries, top_weights, device, update_middle_weights)
    deltas = [collections.OrderedDict() for _ in middles] if with_delta else None
    rest = [k for k in keys if k not in fused]
    if rest:     # the op sequence of the separate calls for the keys the kernel does not take
        _compose(rest, mids, entries, top_weights, top_rates, device, deltas, update_middle_weights)
    fused_set = set(fused)
    # every arrival in one UpdateSlab: pointer rows from slot numbers, once for all keys
    fast = engine.slab_rows([w for e in entries for w, _ in e], fused, {k: top_weights[k].numel() for k in fused},
                            {k: top_weights[k].dtype for k in fused}, device) if fused else None
    for gi, g in enumerate(key_groups if key_groups is not None else [keys]):
        gk = [k for k in g if k in fused_set]
        if gk:
            _fused(gk, mids, entries, top_weights, top_rates, device, deltas, update_middle_weights, fast)
        if after_group is not None:
            after_group(gi)
    if deltas is not None:
        deltas = [collections.OrderedDict((k, d[k]) for k in keys) for d in deltas]
    return top_weights, deltas


def _fusable_keys(keys, mids, entries, top_weights, device, update_middle_weights):
    if len({len(e) for e in entries}) != 1:
        return []
    reps = engine.representatives([w for e in entries for w, _ in e])
    out = []
    for k in keys:
        t = top_weights[k]
        try:
            code = engine.dtype_code(t.dtype)
        except TypeError:
            continue
        if code not in _KERNEL_DTYPES:
            continue
        mw = [w.get(k) for w in mids]
        if any(x is None for x in mw):
            continue
        st = _tiled_stride(mw, t.numel())       # middles contiguous (0) or slots of one tiled store
        if st is None or any(x.dtype != t.dtype or x.device != device for x in mw):
            continue
        tensors = [t] + ([] if st else mw)
        if any(x.dtype != t.dtype or x.numel() != t.numel() or x.device != device
               or not x.is_contiguous() for x in tensors):
            continue
        if any(k not in w or engine.weight_dtype(w, k) != t.dtype for w in reps):
            continue
        if update_middle_weights and len({w[k].data_ptr() for w in mids}) != len(mids):
            continue   # middles updated in place must not share a tensor
        out.append(k)
    return out


def _fused(keys, mids, entries, top_weights, top_rates, device, deltas, update_middle_weights, fast=None):
    """``fast``: slab pointer rows of every key (engine.slab_rows) or None (per-view rows)."""
    keep = []
    mid_rates = [[r for _, r in e] for e in entries]
    groups = collections.OrderedDict()
    for k in keys:
        groups.setdefault(engine.dtype_code(top_weights[k].dtype), []).append(k)
    for code, ks in groups.items():
        segs = []
        for k in ks:
            t = top_weights[k]
            ptrs, stride = [], None
            ok = True
            for e in (entries if fast is None else ()):
                row, ts = engine._client_row([w[k] for w, _ in e], t, device, keep)
                if stride is None:
                    stride = ts
                elif ts != stride:     # mixed tiled / contiguous middles: contiguous copies
                    ok = False
                    break
                ptrs.extend(row)
            if fast is not None:
                ptrs, stride = fast[k]
            elif not ok:
                ptrs, stride = [], 0
                for e in entries:
                    for w, _ in e:
                        c = engine.logical_tensor(w, k).reshape(-1).to(device).contiguous()
                        keep.append(c)
                        ptrs.append(c.data_ptr())
            d_ptrs = None
            if deltas is not None:
                for d in deltas:
                    d[k] = torch.empty_like(t)
                d_ptrs = [d[k].data_ptr() for d in deltas]
            segs.append(engine.HierSeg(numel=t.numel(), mid_w=[w[k].data_ptr() for w in mids],
                                       clients=np.asarray(ptrs, dtype=np.uint64), mid_delta=d_ptrs,
                                       top_in=t.data_ptr(), top_out=t.data_ptr(), tile_stride=stride,
                                       mid_tile_stride=_tiled_stride([w[k] for w in mids], t.numel())))
        engine.hier_fedbuff_(segs, code, mid_rates, [1] * len(mids), top_rates, top_accum=True, top_goal=None,
                             device=device, keep=keep, mid_readonly=not update_middle_weights, sync=True)
    engine._keepalive(keep, device)


def _compose(keys, mids, entries, top_weights, top_rates, device, deltas, update_middle_weights):
    """The reference's op sequence for ``keys``: FedAvg per middle (kernel), delta
    (common/util.py:152-159, a flame_elementwise program), FedAvg of the deltas at the top
    (kernel)."""
    top_entries = []
    for i, (w, e) in enumerate(zip(mids, entries)):
        lw = {k: engine.logical_tensor(w, k) for k in keys}      # slab-slot middles: logical copies
        new = {k: lw[k].clone() for k in keys}                   # deepcopy(self.weights)
        engine.accumulate(new, [({k: x[k] for k in keys}, r) for x, r in e], device=device)
        d = {k: ew.materialize(ew.Lazy.of(new[k]) - ew.Lazy.of(lw[k]), device=device)[0] for k in keys}
        if update_middle_weights:
            for k in keys:
                if lw[k] is w[k]:
                    w[k].copy_(new[k])
                else:
                    _write_tiled(w[k], new[k])
        if deltas is not None:
            deltas[i].update(d)
        top_entries.append((d, top_rates[i]))
    engine.accumulate({k: top_weights[k] for k in keys}, top_entries, device=device)
