"""FedDyn -- drop-in for lib/python/flame/optimizer/feddyn.py:31-139.

Server side of FedDyn (caller: mode/horizontal/feddyn/top_aggregator.py:101-163):
``do()`` is FedAvg with uniform rate ``1/len(cache)`` (:96-103, FedAvg kernel),
the per-trainer history ``h_end += w_end`` (``add_to_hist`` :125-139), the mean
history ``Σ_end (1/len(hist)) * h_end`` over ends that have one (:105-112) and
``cld_model = avg + mean`` (:113).  Every one of those is the same weighted
client reduction, so each is ONE ``flame_agg_reduce`` launch per dtype over
all keys (and, for the history, over all arriving ends), bit-identical to the
reference's torch-CPU op sequence.  Keys whose dtypes mix (int buffers, whose
``rate * h`` the reference promotes to fp32) follow the reference ops with
torch on the device.

History tensors are private device copies: the reference aliases the first
update it sees for an end (``local_param_dict[end] = tres.weights``) and then
rebinds to new tensors on every add; copying once lets later adds run in place
without ever touching the caller's (or an UpdateSlab slot's) memory.
"""
import collections
import logging

import torch

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
        entries, arrivals = [], []
        for k in list(cache.iterkeys()):
            tres = cache.pop(k)
            arrivals.append((k, tres.weights))
            entries.append((tres.weights, rate))
        device = engine.pick_device(base_weights, *[w for w, _ in entries])
        self._add_to_hist(arrivals, device)
        engine.accumulate(self.agg_weights, entries, device=device)
        avg_model = self.agg_weights
        self.cld_model = self._cld(avg_model, device)
        return avg_model

    # ------------------------------------------------------------------ history
    def _add_to_hist(self, arrivals, device):
        """h_end = h_end + w_end for tracked ends (one launch per dtype), copies for new ones."""
        outs, clients = [], []
        for end, w in arrivals:
            h = self.local_param_dict.get(end)
            if h is None:
                if end not in self.local_param_dict:
                    logger.debug(f"adding untracked end {end} to hist terms")
                self.local_param_dict[end] = {k: _own_copy(w, k, device) for k in w.keys()}
                continue
            for k, v in h.items():
                if v.dtype == w[k].dtype and v.is_floating_point():
                    outs.append(v)
                    clients.append([w[k]])
                else:  # reference op (keeps its dtype promotion)
                    h[k] = v + engine.logical_tensor(w, k).to(v.device)
        if outs:
            engine.reduce_(outs, outs, clients, [1.0])

    def _cld(self, avg_model, device):
        """{k: avg[k] + (0.0 + Σ_end rate*h_end[k])}, rate = 1/len(local_param_dict) (feddyn.py:105-113)."""
        hist = [h for h in self.local_param_dict.values() if h is not None]
        rate = 1 / len(self.local_param_dict)
        cld = {}
        fast = [k for k in avg_model
                if avg_model[k].is_floating_point() and all(h[k].dtype == avg_model[k].dtype for h in hist)]
        if fast:
            avg = [engine._Target(avg_model[k], device).dev for k in fast]
            # the zero start reproduces `0.0 + rate*h` (a -0.0 product becomes +0.0)
            means = [torch.zeros(a.numel(), dtype=a.dtype, device=device) for a in avg]
            if hist:
                engine.reduce_(means, means, [[h[k] for h in hist] for k in fast], [rate] * len(hist))
            outs = [torch.empty_like(a) for a in avg]
            engine.reduce_(outs, avg, [[m] for m in means], [1.0])
            for k, o in zip(fast, outs):
                cld[k] = o if avg_model[k].device == device else o.to(avg_model[k].device)
        for k in avg_model:
            if k in cld:
                continue
            a = avg_model[k]
            mean = 0.0
            for h in hist:   # reference ops (int history: rate*h promotes to fp32)
                mean = mean + rate * h[k]
            cld[k] = (a.to(device) + mean).to(a.device)
        return {k: cld[k] for k in avg_model}


def _own_copy(weights, k, device):
    """A private contiguous device copy of weights[k] in its logical shape."""
    return engine.logical_tensor(weights, k).to(device, copy=True).contiguous()
