"""FedBuff on MI355X -- drop-in for lib/python/flame/optimizer/fedbuff.py:38-157.

Same contract: ``rate = 1/math.sqrt(1 + version - tres.version)`` computed in
Python (so stale-version errors raise exactly as in the reference, :96); with
``agg_goal_weights is None`` each cached entry re-creates the aggregate
(:139-140,154-155), so only the last entry of that call survives (reference
quirk, kept); otherwise ``agg[k] += tmp`` in place.  ``scale_add_agg_weights``
mutates and returns ``base_weights`` (:122-127); integer tensors raise like
torch's ``int += float`` does.
"""
import logging
import math

from .. import engine
from .abstract import AbstractOptimizer
from .regularizer import Regularizer

logger = logging.getLogger(__name__)


class FedBuff(AbstractOptimizer):
    """FedBuff class."""

    def __init__(self):
        self.agg_goal_weights = None
        self.is_agg_weights_none = True
        self.regularizer = Regularizer()

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

    def _apply(self, entries):
        if not entries:
            return
        if self.is_agg_weights_none:
            weights, rate = entries[-1]
            self.agg_goal_weights = engine.first_tmp(weights, rate)
        else:
            engine.accumulate(self.agg_goal_weights, entries)

    def scale_add_agg_weights(self, base_weights, agg_goal_weights, agg_goal: int):
        """base[k] += agg[k] / agg_goal in place; returns base_weights (fedbuff.py:101-127)."""
        return self._scale_add(base_weights, agg_goal_weights, agg_goal, None)

    def scale_add_agg_weights_with_delta(self, base_weights, agg_goal_weights, agg_goal: int):
        """scale_add fused with the middle aggregator's upload delta (new - old).

        Equals ``prev = deepcopy(w); scale_add(w, ...); delta_weights_pytorch(w, prev)``
        (asyncfl/middle_aggregator.py:221-226,246; common/util.py:152-159) in one pass.
        Returns ``(base_weights, delta)``.
        """
        import torch
        device = engine.pick_device(base_weights, agg_goal_weights)
        delta = {k: torch.empty(base_weights[k].shape, dtype=base_weights[k].dtype, device=device)
                 for k in base_weights.keys()}
        return self._scale_add(base_weights, agg_goal_weights, agg_goal, delta), delta

    def _scale_add(self, base_weights, agg_goal_weights, agg_goal, delta):
        keys = list(base_weights.keys())
        device = engine.pick_device(base_weights, agg_goal_weights)
        targets = [engine._Target(base_weights[k], device) for k in keys]
        engine.scale_add_([t.dev for t in targets], [agg_goal_weights[k] for k in keys], agg_goal,
                          [delta[k] for k in keys] if delta is not None else None)
        for t in targets:
            t.writeback()
        return base_weights
