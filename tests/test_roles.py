"""The role-side cache binding (flame_amd.roles): a role whose internal_init creates
diskcache caches exactly as flame's do (syncfl/top_aggregator.py:91-95,
scaffold/top_aggregator.py:66-69) gets DeviceUpdateCache objects, and the calls the
roles and optimizers make on them behave as on diskcache."""
import importlib.util
import os

import torch

import scenarios as S

_SHIM = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "_shim", "diskcache.py")


def _disk_cache_cls():
    spec = importlib.util.spec_from_file_location("_diskcache_shim", _SHIM)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.Cache


def test_patched_role_gets_device_cache_and_replays_role_calls():
    from flame_amd import roles
    from flame_amd.ingest import DeviceUpdateCache
    Cache = _disk_cache_cls()

    class Role:                                 # syncfl TopAggregator.internal_init, cache part
        def internal_init(self):
            self.cache = Cache()
            self.cache.reset("size_limit", 1e15)
            self.cache.reset("cull_limit", 0)

    class ScaffoldRole(Role):                   # scaffold/top_aggregator.py:64-69
        def internal_init(self):
            super().internal_init()
            self.control_cache = Cache()
            self.control_cache.reset("size_limit", 1e15)
            self.control_cache.reset("cull_limit", 0)

    roles.patch_role_class(Role, placement="host")
    roles.patch_role_class(Role, placement="host")          # idempotent
    roles.patch_role_class(ScaffoldRole, placement="host")
    r = Role()
    r.internal_init()
    assert isinstance(r.cache, DeviceUpdateCache)
    assert r.cache.reset("size_limit", 1e15) is None and r.cache.reset("cull_limit", 0) is None
    g = torch.Generator().manual_seed(1)
    ups = {f"end{i}": {"w": torch.randn(5, generator=g)} for i in (3, 1, 2)}
    for e, w in ups.items():                    # syncfl/top_aggregator.py:154-156
        r.cache[e] = S.TR(w, 10)
    assert len(r.cache) == 3 and "end1" in r.cache
    assert list(r.cache.iterkeys()) == ["end1", "end2", "end3"]        # diskcache key order
    t = r.cache.pop("end2")
    assert torch.equal(t.weights["w"], ups["end2"]["w"]) and len(r.cache) == 2
    assert r.cache.pop("nope") is None

    s = ScaffoldRole()
    s.internal_init()
    assert isinstance(s.cache, DeviceUpdateCache) and isinstance(s.control_cache, DeviceUpdateCache)


def test_install_cache_moves_entries_in_order():
    from flame_amd import roles
    from flame_amd.ingest import DeviceUpdateCache
    Cache = _disk_cache_cls()

    class R:
        pass
    r = R()
    r.cache = Cache()
    for e in ("b", "a", "c"):
        r.cache[e] = S.TR({"w": torch.full((3,), float(ord(e)))}, 1)
    out = roles.install_cache(r, placement="host")
    assert out is r.cache and isinstance(out, DeviceUpdateCache)
    assert list(out.iterkeys()) == ["a", "b", "c"]
    assert float(out.pop("c").weights["w"][0]) == float(ord("c"))
    assert roles.install_cache(r, placement="host") is out                # already device-resident


def test_install_device_cache_skips_unimportable_roles():
    from flame_amd import roles
    # flame's role layer does not import in this image (paho, aiostream, ... are absent)
    assert isinstance(roles.install_device_cache(placement="host"), list)


def test_eager_role_patch_enables_batching_after_cache_patch():
    """patch_eager_role_class on a class that inherits internal_init: the parent's cache
    patch (applied before or after) still runs, and the role's flame_amd FedAvg defers;
    FedAvg subclasses (FedOPT) are left alone."""
    from flame_amd import roles
    from flame_amd.ingest import DeviceUpdateCache
    from flame_amd.optimizer import FedAdam, FedAvg
    Cache = _disk_cache_cls()

    class Top:                                  # syncfl TopAggregator.internal_init
        sort = "fedavg"

        def internal_init(self):
            self.cache = Cache()
            self.optimizer = FedAvg() if self.sort == "fedavg" else FedAdam()

    class EagerTop(Top):                        # eager_syncfl/top_aggregator.py: no internal_init
        pass

    roles.patch_eager_role_class(EagerTop)
    roles.patch_eager_role_class(EagerTop)       # idempotent
    roles.patch_role_class(Top, placement="host")
    e = EagerTop()
    e.internal_init()
    assert isinstance(e.cache, DeviceUpdateCache) and e.optimizer.defer is True
    t = Top()
    t.internal_init()
    assert t.optimizer.defer is False            # only the eager role
    EagerTop.sort = "fedadam"
    e2 = EagerTop()
    e2.internal_init()
    # FedOPT keeps FedAvg's own defer off (its FedAvg part runs inside the chain) and queues
    # the round's calls for flame_fedopt_chain instead
    assert e2.optimizer.defer is False and e2.optimizer.chain_defer is True
    Top.sort = "fedadam"
    t2 = Top()
    t2.internal_init()
    assert t2.optimizer.chain_defer is False     # only the eager role
    Top.sort = EagerTop.sort = "fedavg"
    assert isinstance(roles.install_device_cache(eager_batching=True, placement="host"), list)
