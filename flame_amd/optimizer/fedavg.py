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
"""
import logging

from .. import engine
from .abstract import AbstractOptimizer
from .regularizer import Regularizer

logger = logging.getLogger(__name__)


class FedAvg(AbstractOptimizer):
    """FedAvg class."""

    def __init__(self):
        self.agg_weights = None
        self.regularizer = Regularizer()

    def _pop_entries(self, cache, total):
        # after popping, the item is removed from the cache (fedavg.py:80-82); rate = count / total
        return [(tres.weights, tres.count / total) for tres in map(cache.pop, list(cache.iterkeys()))]

    def do(self, base_weights, cache, *, total: int = 0, version: int = 0, **kwargs):
        """Aggregate the cached trainer updates into ``base_weights`` (in place)."""
        logger.debug("calling fedavg (flame_amd)")
        assert base_weights is not None
        self.agg_weights = base_weights
        if len(cache) == 0 or total == 0:
            return None
        entries = self._pop_entries(cache, total)
        # flame_amd.shard passes its plan's waves: one launch per wave, its all-gather started
        # right behind it (callers from flame pass no such kwargs)
        engine.accumulate(self.agg_weights, entries, key_groups=kwargs.get("flame_amd_key_groups"),
                          after_group=kwargs.get("flame_amd_after_group"))
        return self.agg_weights
