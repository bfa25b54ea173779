"""Optimizer ABC -- same contract as lib/python/flame/optimizer/abstract.py:25-36."""
from abc import ABC, abstractmethod


class AbstractOptimizer(ABC):
    """Abstract base class for optimizer implementation."""

    @abstractmethod
    def do(self, base_weights, cache, *, total: int = 0, version: int = 0, **kwargs):
        """Conduct optimization over the cached TrainResults (consumed via cache.pop)."""
