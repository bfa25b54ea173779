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
reference promotes to fp32) follow the reference ops with torch on the device.

History tensors are private device copies: the reference aliases the first
update it sees for an end (``local_param_dict[end] = tres.weights``) and then
rebinds to new tensors on every add; owning them lets later adds run in place
without ever touching the caller's (or an UpdateSlab slot's) memory.
"""
import collections
import logging

import torch

from .. import _native as N
from .. import engine
from .fedavg import FedAvg

logger = logging.getLogger(__name__)

try:  # pragma: no cover - depends on flame being installed
    from flame.optimizer.regularizer.feddyn import FedDynRegularizer  # type: ignore
except Exception:  # noqa: BLE001
    FedDynRegularizer = None


def _is_pre(state) -> bool:
    return getattr(state, "value", state) == "pre"   # flame.common.constants.TrainState.PRE


class FedDyn(FedAvg):
    """FedDyn class."""

    def __init__(self, alpha):
        super().__init__()
        self.alpha = alpha
        self.local_param_dict = dict()
        self.cld_model = None
        if FedDynRegularizer is not None:
            self.regularizer = FedDynRegularizer(self.alpha)

    def save_state(self, state, **kwargs):
        """feddyn.py:51-62: keep history only for the round's active ends (None for new ones)."""
        if _is_pre(state):
            active_ends = kwargs["active_ends"]
            self.local_param_dict = {end: self.local_param_dict.get(end) for end in active_ends}

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
        fused = [k for k in base_weights if self._fusable(k, arrivals, had, device)]
        rest = [k for k in base_weights if k not in fused]
        new_hist = {e: {} for e, _ in arrivals if e not in had}
        cld = {}
        if fused:
            self._fused_round(fused, arrivals, had, rate, device, new_hist, cld)
        if rest:
            self._reference_round(rest, arrivals, had, rate, device, new_hist, cld)
        for e, w in arrivals:
            if e not in had:
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
        """The reference's op sequence with torch on the device (its dtype promotions)."""
        for e, w in arrivals:
            if e in had:
                h = self.local_param_dict[e]
                for k in keys:
                    h[k] = h[k] + engine.logical_tensor(w, k).to(h[k].device)
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
            mean = 0.0
            for h in hist:
                mean = mean + rate_mean * h[k]
            cld[k] = (a.to(device) + mean).to(a.device)


def _own_copy(weights, k, device):
    """A private contiguous device copy of weights[k] in its logical shape."""
    return engine.logical_tensor(weights, k).to(device, copy=True).contiguous()
