"""Role-side binding: the aggregator's update cache.

flame's aggregator roles keep received updates in a disk-backed ``diskcache.Cache``
created in ``internal_init`` (``syncfl/top_aggregator.py:91-95``,
``syncfl/middle_aggregator.py:78-82``; every async / eager / FedDyn / FedGFT role
inherits one of those two, and SCAFFOLD adds a ``control_cache`` the same way,
``scaffold/top_aggregator.py:66-69``).  Each update is then pickled to disk on
``cache[end] = tres`` and unpickled again in the optimizer's ``cache.pop``.

The MI355X path wants those updates in HBM, in the tiled slab the reduction streams at
the read ceiling.  :func:`install_cache` swaps a role's caches for
:class:`flame_amd.ingest.DeviceUpdateCache` objects (same surface: ``reset``,
``__setitem__``, ``__len__``, ``iterkeys``, ``pop``); :func:`patch_role_class` /
:func:`install_device_cache` do it for every instance, by wrapping ``internal_init``,
so flame's own role code is unchanged.  An unpatched role still works with the
drop-in optimizers -- its updates are unpickled into one tensor each (row layout,
16.7 ms instead of 14.8 ms for config 3) after the disk round trip.

The eager top aggregator (``eager_syncfl/top_aggregator.py:36-90``) calls ``do()`` once per
arrival and reads only the object the last call returns; :func:`patch_eager_role_class`
(``install_device_cache(eager_batching=True)``) turns on ``FedAvg(defer=True)`` for it, so
a round's arrivals are reduced in one launch (flame_amd/optimizer/fedavg.py), or, for the
FedOPT family, ``defer=True``: the round's calls run as one flame_fedopt_chain launch.
"""
from __future__ import annotations

import functools
import importlib
import logging

logger = logging.getLogger(__name__)

CACHE_ATTRS = ("cache", "control_cache")

# the classes whose internal_init creates a diskcache.Cache (module, class)
ROLE_CLASSES = (
    ("flame.mode.horizontal.syncfl.top_aggregator", "TopAggregator"),
    ("flame.mode.horizontal.syncfl.middle_aggregator", "MiddleAggregator"),
    ("flame.mode.horizontal.scaffold.top_aggregator", "TopAggregator"),
)


def install_cache(role, *, placement: str = "slab", capacity: int = 256, device=None, shard=None,
                  attrs=CACHE_ATTRS):
    """Replace ``role.cache`` (and ``role.control_cache``) with device-resident caches.

    Call after the role's ``internal_init`` (which creates them).  ``capacity`` is the
    number of slab slots (updates in flight per round: the number of trainers, or the
    async ``aggregation_goal``); an update that finds the slab full is still kept in HBM,
    one allocation per tensor.  ``shard``: a :class:`flame_amd.shard.ShardPlan` -- keep
    only this rank's ranges (parameter-sharded aggregation).  Entries already in a
    replaced cache are moved over in their ``iterkeys()`` order.  Returns ``role.cache``.
    """
    from .ingest import DeviceUpdateCache
    for a in attrs:
        old = getattr(role, a, None)
        if old is None or isinstance(old, DeviceUpdateCache):
            continue
        new = DeviceUpdateCache(device=device, placement=placement, capacity=capacity, shard=shard)
        for k in list(old.iterkeys()):
            new[k] = old.pop(k)
        setattr(role, a, new)
        close = getattr(old, "close", None)
        if callable(close):
            close()
    return getattr(role, "cache", None)


def patch_role_class(cls, **kwargs):
    """Wrap ``cls.internal_init`` so every instance gets device-resident caches right after
    the original runs (idempotent).  ``kwargs`` go to :func:`install_cache`."""
    orig = cls.__dict__.get("internal_init")
    if orig is None or getattr(orig, "_flame_amd_cache", False):
        return cls

    @functools.wraps(orig)
    def internal_init(self, *a, **kw):
        out = orig(self, *a, **kw)
        install_cache(self, **kwargs)
        return out
    internal_init._flame_amd_cache = True
    cls.internal_init = internal_init
    return cls


# the eager aggregators (inherit the syncfl roles' internal_init): one do() per arrival into
# the round's base, only the last result read (eager_syncfl/top_aggregator.py:36-90,
# eager_syncfl/middle_aggregator.py:40-80)
EAGER_ROLE_CLASSES = (
    ("flame.mode.horizontal.eager_syncfl.top_aggregator", "TopAggregator"),
    ("flame.mode.horizontal.eager_syncfl.middle_aggregator", "MiddleAggregator"),
)
EAGER_ROLE_CLASS = EAGER_ROLE_CLASSES[0]


def enable_eager_batching(role):
    """Turn on eager batching for ``role.optimizer``: ``defer=True`` when it is the flame_amd
    FedAvg itself, the queued chain (``FedOPT(defer=True)``: one flame_fedopt_chain launch per
    round) when it is a FedAdam / FedYogi / FedAdaGrad.  Other subclasses (FedProx, FedGFT, ...)
    keep their own ``do``.  Returns whether it was enabled."""
    from .optimizer.fedavg import FedAvg
    from .optimizer.fedopt import FedOPT
    opt = getattr(role, "optimizer", None)
    if type(opt) is FedAvg:
        opt.defer = True
        return True
    if isinstance(opt, FedOPT):
        opt.chain_defer = True
        return True
    return False


def patch_eager_role_class(cls):
    """Wrap ``cls.internal_init`` -- its own, or the one it inherits, looked up at call time
    so a cache patch of the parent still runs -- to call :func:`enable_eager_batching` after
    it (idempotent)."""
    own = cls.__dict__.get("internal_init")
    if getattr(own, "_flame_amd_eager", False):
        return cls

    def internal_init(self, *a, **kw):
        out = own(self, *a, **kw) if own is not None else super(cls, self).internal_init(*a, **kw)
        enable_eager_batching(self)
        return out
    internal_init._flame_amd_eager = True
    internal_init.__doc__ = getattr(own, "__doc__", None)
    cls.internal_init = internal_init
    return cls


def _import_class(mod, name):
    try:
        return getattr(importlib.import_module(mod), name)
    except Exception as e:  # noqa: BLE001  (flame's role layer needs paho, aiostream, ...)
        logger.info("flame_amd.roles: %s.%s not patched (%s)", mod, name, e)
        return None


def install_device_cache(eager_batching: bool = False, **kwargs):
    """Patch flame's aggregator role classes (ROLE_CLASSES) in place; call once before roles
    are composed, next to ``flame_amd.optimizers.install()``.  ``eager_batching``: also
    patch the eager top and middle aggregators (:func:`patch_eager_role_class`).  Returns the patched
    classes; classes whose module does not import here are skipped (logged)."""
    done = []
    for mod, name in ROLE_CLASSES:
        cls = _import_class(mod, name)
        if cls is not None:
            done.append(patch_role_class(cls, **kwargs))
    if eager_batching:
        for mod, name in EAGER_ROLE_CLASSES:
            cls = _import_class(mod, name)
            if cls is not None:
                done.append(patch_eager_role_class(cls))
    return done
