"""Optimizer provider -- mirrors lib/python/flame/optimizers.py:31-48 and
lib/python/flame/object_factory.py:18-29, and installs the MI355X classes into
flame's own provider so existing roles pick them up unchanged.

``OptimizerType`` is a closed enum validated by flame's config
(config.py:55-70,121-123), so the drop-in re-registers the existing keys
(``fedavg``, ``fedadagrad``, ``fedadam``, ``fedyogi``, ``fedbuff``, ``fedprox``,
``feddyn``, ``scaffold``, ``fedgft`` -- every key flame registers) instead of
adding new ones.
"""
from .optimizer import FedAdaGrad, FedAdam, FedAvg, FedBuff, FedDyn, FedGFT, FedProx, FedYogi, Scaffold

DROP_INS = {
    "fedavg": FedAvg,
    "fedadagrad": FedAdaGrad,
    "fedadam": FedAdam,
    "fedyogi": FedYogi,
    "fedbuff": FedBuff,
    "fedprox": FedProx,
    "feddyn": FedDyn,
    "scaffold": Scaffold,
    "fedgft": FedGFT,
}


class ObjectFactory(object):
    """Same semantics as flame.object_factory.ObjectFactory."""

    def __init__(self):
        self._objects = {}

    def register(self, key, obj):
        self._objects[key] = obj

    def create(self, key, **kwargs):
        obj = self._objects.get(key)
        if not obj:
            raise ValueError(key)
        return obj(**kwargs)


class OptimizerProvider(ObjectFactory):
    """Optimizer Provider."""

    def get(self, optimizer_name, **kwargs):
        """Return an optimizer for a given optimizer name."""
        return self.create(optimizer_name, **kwargs)


optimizer_provider = OptimizerProvider()
for _k, _cls in DROP_INS.items():
    optimizer_provider.register(_k, _cls)


def install(provider=None):
    """Re-register flame's optimizer keys with the MI355X classes.

    ``provider`` defaults to ``flame.optimizers.optimizer_provider`` (imported
    lazily; flame must be importable).  Call it once before roles are
    composed, e.g. at the top of an aggregator's ``main.py``.  Returns the
    provider.
    """
    if provider is None:
        from flame.optimizers import optimizer_provider as provider  # type: ignore
        from flame.config import OptimizerType  # type: ignore
        keys = {k: OptimizerType(k) for k in DROP_INS}
    else:
        keys = {k: k for k in DROP_INS}
    for name, cls in DROP_INS.items():
        provider.register(keys[name], cls)
    return provider
