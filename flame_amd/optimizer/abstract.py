"""Optimizer ABC -- same contract as lib/python/flame/optimizer/abstract.py:25-36.

Addition: ``metric_collector`` -- set it to the role's
``MetricCollector`` (``Role.mc``) and the GPU time / HBM rate of every ``do()``
and ``scale_add_agg_weights()`` is saved there (``flame_amd/metrics.py``).
"""
from abc import ABC, abstractmethod

_INSTRUMENTED = ("do", "scale_add_agg_weights", "scale_add_agg_weights_with_delta")


class AbstractOptimizer(ABC):
    """Abstract base class for optimizer implementation."""

    metric_collector = None   # flame MetricCollector (or any object with save(mtype, alias, value))
    metric_alias = None       # key prefix; default: the class name in lower case

    def __init_subclass__(cls, **kwargs):
        super().__init_subclass__(**kwargs)
        from ..metrics import instrument
        for name in _INSTRUMENTED:
            if name in cls.__dict__:
                setattr(cls, name, instrument(cls.__dict__[name]))

    @abstractmethod
    def do(self, base_weights, cache, *, total: int = 0, version: int = 0, **kwargs):
        """Conduct optimization over the cached TrainResults (consumed via cache.pop)."""
