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
promotes to fp32 in this step, and any key whose dtype changed) are reduced by
the FedAvg kernel and then follow the reference op sequence with torch ops on
the device.

Ownership: ``base_weights`` is mutated in place into the
FedAvg result (``self.agg_weights``); ``m_t``/``v_t`` persist across rounds on
the device; each round returns a NEW OrderedDict of new tensors, like the
reference.  ``d_t`` is not materialised by the fused path; it is computed
lazily from ``agg_weights`` and the previous ``current_weights`` on access.
"""
import logging
import os
from abc import abstractmethod
from collections import OrderedDict

import torch

from .. import engine
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

    def __init__(self, beta_1, beta_2, eta, tau):
        super().__init__()
        self.current_weights = None
        self._d_t = None
        self._prev_current = None
        self.m_t = None
        self.v_t = None
        self.beta_1 = beta_1
        self.beta_2 = beta_2
        self.eta = eta
        self.tau = tau

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

    def _adapt_generic(self, keys, average, current, state_zero):
        """fedopt.py:106-129 op sequence (torch ops on the device) for non-fp32 keys."""
        out = {}
        for k in keys:
            d = average[k] - current[k]
            m = torch.zeros_like(d) if state_zero or k not in self.m_t else self.m_t[k]
            m = self.beta_1 * m + (1 - self.beta_1) * d
            v = torch.zeros_like(d) if state_zero or k not in self.v_t else self.v_t[k]
            v = self._delta_v_tensor(v, d)
            self.m_t[k], self.v_t[k] = m, v
            sq = torch.sqrt(v)
            # torch-CPU adds a Python scalar to a bf16/fp16 tensor after rounding the scalar
            # to that dtype (unlike mul/div, which use it in fp32); GPU torch keeps it fp32.
            tau = float(torch.tensor(self.tau, dtype=sq.dtype)) if sq.dtype in (torch.bfloat16, torch.float16) \
                else self.tau
            out[k] = current[k] + self.eta * m / (sq + tau)
        return out

    @abstractmethod
    def _delta_v_tensor(self, v, d):
        """The subclass's _delta_v_pytorch for one key."""
