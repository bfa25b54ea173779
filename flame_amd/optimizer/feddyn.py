"""FedDyn -- drop-in for lib/python/flame/optimizer/feddyn.py:31-139.

Server side of FedDyn (caller: mode/horizontal/feddyn/top_aggregator.py:101-163):
``do()`` is FedAvg with uniform rate ``1/len(cache)`` (:96-103), the per-trainer
history ``h_end += w_end`` (``add_to_hist`` :125-139), the mean history
``0.0 + Σ_end (1/len(hist)) * h_end`` over ends that have one (:105-112) and
``cld_model = avg + mean`` (:113).  Float keys whose average, updates and
histories share one dtype run as ONE ``flame_feddyn_round`` launch per dtype
(``engine.feddyn_program``): each update and history is read once and each
updated history written once, instead of the reference's four passes (history,
average, mean, cld).  The average sums in cache order and the mean in
``local_param_dict`` order, each op rounded as torch-CPU rounds it, so results
are bit-identical.  Keys whose dtypes mix (int buffers, whose ``rate * h`` the
reference promotes to fp32) run the reference's statements as ``flame_elementwise``
programs (``flame_amd.elementwise``: torch's promotions, torch-CPU's arithmetic).

History tensors are private device copies: the reference aliases the first
update it sees for an end (``local_param_dict[end] = tres.weights``) and then
rebinds to new tensors on every add; owning them lets later adds run in place
without ever touching the caller's (or an UpdateSlab slot's) memory.

``history="pingpong"``: the fused keys' histories live in two tiled stores
(:class:`_PingPongHistories`, the UpdateSlab layout: one contiguous
``[ends][chunk]`` block per chunk) and an arrival's updated history ``h + w`` is
written to the OTHER store -- a round never writes the addresses it reads, and each
workgroup streams one contiguous history block.  Opt-in: measured through the drop-in at
512 ends x 16M fp32 it is SLOWER than the in-place per-end rows (tiled ping-pong 17.75 ms,
row ping-pong 17.13 ms, rows 16.95 ms; DESIGN.md §4, profiles/r02_feddyn_history_ab.log),
for twice the history memory; round 1's 12.5M-param probe had suggested a gain.
"""
import collections
import collections.abc
import logging

import torch

from .. import _native as N
from .. import elementwise as ew, engine
from .fedavg import FedAvg

logger = logging.getLogger(__name__)

try:  # pragma: no cover - depends on flame being installed
    from flame.optimizer.regularizer.feddyn import FedDynRegularizer  # type: ignore
except Exception:  # noqa: BLE001
    FedDynRegularizer = None


def _is_pre(state) -> bool:
    return getattr(state, "value", state) == "pre"   # flame.common.constants.TrainState.PRE


class _PingPongHistories:
    """Per-end FedDyn histories of the fused keys in two stores.  ``cur[end]`` names the
    store holding an end's current history; a round reads ``cur`` and writes ``1 - cur``
    (then flips it).  ``tiled``: each store is one UpdateSlab (an end = one slot index in
    both); else every end owns two contiguous tensors per key."""

    def __init__(self, template, device, capacity, tiled=True):
        from ..slab import UpdateSlab
        self.template = template
        self.device = device
        self.capacity = capacity
        self.tiled = tiled
        self.stores = [UpdateSlab(template, capacity, device), UpdateSlab(template, capacity, device)] if tiled \
            else None
        self.rows = {}            # untiled: end -> ({k: tensor}, {k: tensor})
        self.slot, self.cur = {}, {}
        self.free = list(range(capacity - 1, -1, -1))

    def keys(self):
        return list(self.template.keys())

    def ensure(self, ends):
        need = list(dict.fromkeys(e for e in ends if e not in self.slot))
        if not self.tiled:
            for e in need:
                self.slot[e] = 0
                self.cur[e] = 0
                self.rows[e] = tuple({k: torch.empty(t.shape, dtype=t.dtype, device=self.device)
                                      for k, t in self.template.items()} for _ in range(2))
            return
        if len(need) > len(self.free):
            self._grow(len(self.slot) + len(need))
        for e in need:
            self.slot[e] = self.free.pop()
            self.cur[e] = 0

    def release(self, keep):
        for e in [e for e in self.slot if e not in keep]:
            s = self.slot.pop(e)
            self.cur.pop(e)
            if self.tiled:
                self.free.append(s)
            else:
                self.rows.pop(e)

    def _grow(self, need):
        old = self.stores
        cap = max(need, 2 * self.capacity)
        from ..slab import UpdateSlab
        self.stores = [UpdateSlab(self.template, cap, self.device), UpdateSlab(self.template, cap, self.device)]
        for e, s in self.slot.items():
            c = self.cur[e]
            for k in self.template:
                self.stores[c].slot_view(s, k).copy_(old[c].slot_view(s, k))
        self.free = list(range(cap - 1, self.capacity - 1, -1)) + self.free
        self.capacity = cap

    def ptr(self, store, k, end) -> int:
        if not self.tiled:
            return self.rows[end][store][k].data_ptr()
        _, _, base, slot_bytes, _ = self.stores[store].key_layout(k)
        return base + self.slot[end] * slot_bytes

    def write(self, end, k, h) -> None:
        """``h`` (the end's whole history of key ``k``) into the store holding its current one."""
        if not self.tiled:
            self.rows[end][self.cur[end]][k].copy_(h.reshape(self.rows[end][self.cur[end]][k].shape))
        else:
            self.stores[self.cur[end]].write_key(self.slot[end], k, h.reshape(-1))

    def tile_stride(self, k) -> int:
        return self.stores[0].key_layout(k)[4] if self.tiled else 0

    def read(self, end, k):
        """The end's current history of key ``k`` (a contiguous copy in the model's shape)."""
        if not self.tiled:
            return self.rows[end][self.cur[end]][k].clone()
        st = self.stores[self.cur[end]]
        return st.read(self.slot[end], k)


class _StoredHistory(collections.abc.MutableMapping):
    """``local_param_dict[end]`` under ``history="pingpong"``: the fused keys read from the
    ping-pong stores (copies, on access), the other keys are plain tensors (``rest``)."""

    def __init__(self, store, end, order, rest):
        self._store, self._end, self._order, self.rest = store, end, list(order), dict(rest)

    def __getitem__(self, k):
        if k in self.rest:
            return self.rest[k]
        if k in self._store.template and k in self._order:
            return self._store.read(self._end, k)
        raise KeyError(k)

    def __setitem__(self, k, v):
        self.rest[k] = v
        if k not in self._order:
            self._order.append(k)

    def __delitem__(self, k):
        raise TypeError("FedDyn history keys are fixed")

    def __iter__(self):
        return iter(self._order)

    def __len__(self):
        return len(self._order)


class FedDyn(FedAvg):
    """FedDyn class."""

    def __init__(self, alpha, history: str = "rows"):
        super().__init__()
        if history not in ("rows", "pingpong", "pingpong_rows"):
            raise ValueError("history must be 'rows', 'pingpong' or 'pingpong_rows'")
        self.alpha = alpha
        self.local_param_dict = dict()
        self.cld_model = None
        self.history = history
        self._pp = None
        if FedDynRegularizer is not None:
            self.regularizer = FedDynRegularizer(self.alpha)

    def save_state(self, state, **kwargs):
        """feddyn.py:51-62: keep history only for the round's active ends (None for new ones)."""
        if _is_pre(state):
            active_ends = kwargs["active_ends"]
            self.local_param_dict = {end: self.local_param_dict.get(end) for end in active_ends}
            if self._pp is not None:
                self._pp.release({e for e, h in self.local_param_dict.items() if h is not None})

    def do(self, base_weights, cache, *, total: int = 0, version: int = 0, **kwargs):
        logger.debug("calling feddyn (flame_amd)")
        assert base_weights is not None
        self.agg_weights = base_weights
        if len(cache) == 0 or total == 0:
            return None
        rate = 1 / len(cache)
        arrivals = []
        for k in list(cache.iterkeys()):
            tres = cache.pop(k)
            arrivals.append((k, tres.weights))
        device = engine.pick_device(base_weights, *[w for _, w in arrivals])
        had = {e for e, h in self.local_param_dict.items() if h is not None}
        for end, _ in arrivals:     # add_to_hist appends untracked ends in arrival order (:135-139)
            if end not in self.local_param_dict:
                logger.debug(f"adding untracked end {end} to hist terms")
                self.local_param_dict[end] = None
        pp = self.history.startswith("pingpong")
        if pp and self._pp is None:
            self._init_pingpong(arrivals, device)
        # keys some end's history of which left the stores (one pass over the ends, not one per key)
        moved = set()
        if pp:
            for h in self.local_param_dict.values():
                if isinstance(h, _StoredHistory) and h.rest:
                    moved.update(h.rest.keys())
        fused = [k for k in base_weights if (self._fusable_pp(k, arrivals, moved) if pp
                                             else self._fusable(k, arrivals, had, device))]
        rest = [k for k in base_weights if k not in fused]
        new_hist = {e: {} for e, _ in arrivals if e not in had}
        cld = {}
        if pp:
            # the reference-path keys first: they read the histories from the store holding
            # them before the fused round flips the arriving ends to the other store; their
            # updated histories then join that store (_pp_absorb)
            if rest:
                self._reference_round(rest, arrivals, had, rate, device, new_hist, cld)
            if fused:
                self._fused_round_pp(fused, arrivals, had, rate, device, cld)
            if rest:
                self._pp_absorb(rest, arrivals, had, new_hist)
        else:
            if fused:
                self._fused_round(fused, arrivals, had, rate, device, new_hist, cld)
            if rest:
                self._reference_round(rest, arrivals, had, rate, device, new_hist, cld)
        for e, w in arrivals:
            if e not in had:
                if pp:
                    self.local_param_dict[e] = _StoredHistory(self._pp, e, w.keys(),
                                                              {k: new_hist[e][k] for k in w.keys()
                                                               if k in rest and k in new_hist[e]})
                else:
                    self.local_param_dict[e] = {k: new_hist[e][k] for k in w.keys()}
        avg_model = self.agg_weights
        self.cld_model = {k: cld[k] for k in avg_model}
        return avg_model

    def _fusable(self, k, arrivals, had, device) -> bool:
        a = self.agg_weights[k]
        if not a.is_floating_point():
            return False
        for _, w in arrivals:
            if k not in w or w[k].dtype != a.dtype:
                return False
        for e in had:
            h = self.local_param_dict[e].get(k)
            if (h is None or h.dtype != a.dtype or h.device != device or not h.is_contiguous()
                    or h.numel() != a.numel()):
                return False
        return True

    # ------------------------------------------------------------------ ping-pong histories
    def _init_pingpong(self, arrivals, device):
        """The fused keys (float, every arrival in the aggregate's dtype) at the first round
        become the stores' template; capacity = the round's ends (grown when more join)."""
        keys = [k for k, a in self.agg_weights.items()
                if a.is_floating_point() and all(k in w and w[k].dtype == a.dtype for _, w in arrivals)]
        template = collections.OrderedDict((k, torch.empty(self.agg_weights[k].shape, dtype=self.agg_weights[k].dtype,
                                                           device="meta")) for k in keys)
        self._pp = _PingPongHistories(template, device, max(len(self.local_param_dict), 1),
                                      tiled=self.history == "pingpong")

    def _fusable_pp(self, k, arrivals, moved) -> bool:
        a = self.agg_weights[k]
        t = self._pp.template.get(k)
        if t is None or t.dtype != a.dtype or t.shape != a.shape:
            return False
        if not all(k in w and engine.weight_dtype(w, k) == a.dtype for _, w in arrivals):
            return False
        # an end whose history of k left the stores (another dtype, see _pp_absorb) keeps the
        # key on the reference path: the stores do not hold its current value
        return k not in moved

    def _pp_absorb(self, keys, arrivals, had, new_hist):
        """Template keys that took the reference path this round (an arrival in another dtype):
        each arriving end's updated history goes back into the store holding its current one
        -- a new end gets its slot -- so a later fused round reads the right bytes.  A history
        whose dtype or size no longer fits the store (torch promoted it) stays in the end's
        ``rest`` and the key off the fused path (_fusable_pp)."""
        pp = self._pp
        tk = [k for k in keys if k in pp.template]
        if not tk:
            return
        pp.ensure([e for e, _ in arrivals])
        for e, _ in arrivals:
            for k in tk:
                src = new_hist[e] if e not in had else self.local_param_dict[e].rest
                h = src.get(k)
                t = pp.template[k]
                if h is None or h.dtype != t.dtype or h.numel() != t.numel() or not h.is_cuda:
                    continue
                pp.write(e, k, h)
                del src[k]

    def _fused_round_pp(self, keys, arrivals, had, rate, device, cld):
        pp = self._pp
        steps, n_phase1 = engine.feddyn_program([e for e, _ in arrivals], list(self.local_param_dict), had)
        pp.ensure([e for _, e in steps])
        flags = [f for f, _ in steps]
        rate_mean = 1 / len(self.local_param_dict)
        wmap = dict(arrivals)
        w_ends = [e for f, e in steps if f & N.FLAME_DYN_W]
        targets = {k: engine._Target(self.agg_weights[k], device) for k in keys}
        groups = collections.OrderedDict()
        for k in keys:
            groups.setdefault(engine.dtype_code(self.agg_weights[k].dtype), []).append(k)
        keep = []
        for code, ks in groups.items():
            segs = []
            for k in ks:
                t = targets[k].dev
                row, tile_stride = engine._client_row([wmap[e][k] for e in w_ends], t, device, keep)
                wptr = dict(zip(w_ends, row))
                c = torch.empty_like(t)
                cld[k] = c
                written = set()
                ptrs = []
                for f, e in steps:
                    # h is read from the store holding the end's history (the one just written,
                    # if a phase-1 step of this program wrote it); h' goes to the other store
                    src = pp.cur[e] ^ (1 if e in written else 0)
                    ptrs.append((wptr[e] if f & N.FLAME_DYN_W else 0,
                                 pp.ptr(src, k, e) if f & N.FLAME_DYN_HIN else 0,
                                 pp.ptr(pp.cur[e] ^ 1, k, e) if f & N.FLAME_DYN_HOUT else 0))
                    if f & N.FLAME_DYN_HOUT:
                        written.add(e)
                segs.append(engine.DynSeg(t.numel(), out=t.data_ptr(), inp=t.data_ptr(), cld=c.data_ptr(),
                                          steps=ptrs, tile_stride=tile_stride, hist_tile_stride=pp.tile_stride(k)))
            engine.feddyn_round_(code, segs, flags, n_phase1, rate, rate_mean, device, keep)
        for f, e in steps:
            if f & N.FLAME_DYN_HOUT:
                pp.cur[e] ^= 1
        engine._keepalive(keep, device)
        for k, t in targets.items():
            t.writeback()
            a = self.agg_weights[k]
            if a.device != device:
                cld[k] = cld[k].to(a.device)
            cld[k] = cld[k].view(a.shape)

    # ------------------------------------------------------------------ one launch per dtype
    def _fused_round(self, keys, arrivals, had, rate, device, new_hist, cld):
        steps, n_phase1 = engine.feddyn_program([e for e, _ in arrivals], list(self.local_param_dict), had)
        flags = [f for f, _ in steps]
        rate_mean = 1 / len(self.local_param_dict)
        wmap = dict(arrivals)
        w_ends = [e for f, e in steps if f & N.FLAME_DYN_W]
        targets = {k: engine._Target(self.agg_weights[k], device) for k in keys}
        groups = collections.OrderedDict()
        for k in keys:
            groups.setdefault(engine.dtype_code(self.agg_weights[k].dtype), []).append(k)
        keep = []
        for code, ks in groups.items():
            segs = []
            for k in ks:
                t = targets[k].dev
                hbuf = {}
                for f, e in steps:
                    if e in had:
                        hbuf[e] = self.local_param_dict[e][k]
                    elif e not in hbuf:   # first history of this end: the kernel writes w into it
                        hbuf[e] = new_hist[e][k] = torch.empty(engine.logical_shape(wmap[e], k), dtype=t.dtype,
                                                               device=device)
                row, tile_stride = engine._client_row([wmap[e][k] for e in w_ends], t, device, keep)
                wptr = dict(zip(w_ends, row))
                c = torch.empty_like(t)
                cld[k] = c
                ptrs = [(wptr[e] if f & N.FLAME_DYN_W else 0,
                         hbuf[e].data_ptr() if f & N.FLAME_DYN_HIN else 0,
                         hbuf[e].data_ptr() if f & N.FLAME_DYN_HOUT else 0) for f, e in steps]
                segs.append(engine.DynSeg(t.numel(), out=t.data_ptr(), inp=t.data_ptr(), cld=c.data_ptr(),
                                          steps=ptrs, tile_stride=tile_stride))
            engine.feddyn_round_(code, segs, flags, n_phase1, rate, rate_mean, device, keep)
        engine._keepalive(keep, device)
        for k, t in targets.items():
            t.writeback()
            a = self.agg_weights[k]
            if a.device != device:
                cld[k] = cld[k].to(a.device)
            cld[k] = cld[k].view(a.shape)

    # ------------------------------------------------------------------ mixed-dtype keys
    def _reference_round(self, keys, arrivals, had, rate, device, new_hist, cld):
        """The reference's statements (feddyn.py:90-113,125-139) for the mixed-dtype keys, with
        torch's dtype promotions: each one recorded on elementwise.Lazy operands and run as a
        flame_elementwise program on ``device`` (the mean of the histories in launches of up
        to _MEAN_TERMS terms); the FedAvg part through engine.accumulate."""
        for e, w in arrivals:
            if e in had:
                h = self.local_param_dict[e]
                for k in keys:
                    s = ew.materialize(ew.Lazy.of(h[k]) + ew.Lazy.of(engine.logical_tensor(w, k)), device=device)[0]
                    h[k] = s if h[k].device == device else s.to(h[k].device)
            else:
                for k in keys:
                    new_hist[e][k] = _own_copy(w, k, device)
        engine.accumulate({k: self.agg_weights[k] for k in keys},
                          [({k: w[k] for k in keys}, rate) for _, w in arrivals], device=device)
        rate_mean = 1 / len(self.local_param_dict)
        hist = [new_hist[e] if e in new_hist else h for e, h in self.local_param_dict.items()
                if h is not None or e in new_hist]
        for k in keys:
            a = self.agg_weights[k]
            mean, terms = 0.0, 0          # mean = 0.0; mean = mean + rate_mean * h[k] per history
            for h in hist:
                mean = mean + rate_mean * ew.Lazy.of(h[k])
                terms += 1
                if terms == _MEAN_TERMS:
                    mean, terms = ew.Lazy.of(ew.materialize(mean, device=device)[0]), 0
            c = ew.materialize(ew.Lazy.of(a) + mean, device=device)[0]
            cld[k] = c if a.device == device else c.to(a.device)


_MEAN_TERMS = 8      # histories per flame_elementwise launch of the mean (<= 6 ops each; 64 per program)


def _own_copy(weights, k, device):
    """A private contiguous device copy of weights[k] in its logical shape."""
    return engine.logical_tensor(weights, k).to(device, copy=True).contiguous()
