"""Child process of tests/test_env_classes.py::test_install_into_flame_provider.

flame is importable here (the reference tree + the diskcache shim on PYTHONPATH).  Calls
``flame_amd.optimizers.install()`` with no argument -- the branch that imports
``flame.optimizers.optimizer_provider`` and ``flame.config.OptimizerType``
(lib/python/flame/optimizers.py:39-48, config.py:55-70) -- and then resolves optimizers the
way flame's roles do: ``optimizer_provider.get(self.config.optimizer.sort,
**self.config.optimizer.kwargs)`` (mode/horizontal/syncfl/top_aggregator.py:97-99) on a job's
optimizer block parsed by flame's own pydantic ``Optimizer`` model (config.py:121-123).  Prints
one JSON line."""
import json
import sys

sys.path.insert(0, sys.argv[1])            # the repository root


def main():
    import torch  # noqa: F401  (flame detects the ML framework from the imported modules, common/util.py)
    from flame.config import Config, OptimizerType
    from flame.optimizers import optimizer_provider

    out = {"before": {}, "after": {}, "config": {}}
    kw = {"fedavg": {}, "fedadam": {"beta_1": 0.8}, "fedyogi": {"eta": 0.05}, "fedadagrad": {"tau": 1e-4},
          "fedbuff": {}, "fedprox": {"mu": 0.01}, "feddyn": {"alpha": 0.01}, "scaffold": {"k": 3},
          "fedgft": {"fair": "SP", "gamma": 0.5}}
    for t in OptimizerType:
        o = optimizer_provider.get(t, **kw[t.value])
        out["before"][t.value] = type(o).__module__ + "." + type(o).__name__

    import flame_amd.optimizers as fo
    ret = fo.install()
    out["returned_flame_provider"] = ret is optimizer_provider
    for t in OptimizerType:
        o = optimizer_provider.get(t, **kw[t.value])
        o2 = optimizer_provider.get(t.value, **kw[t.value])       # a plain str key resolves the same
        out["after"][t.value] = {"cls": type(o).__module__ + "." + type(o).__name__,
                                 "same_as_drop_in": type(o) is fo.DROP_INS[t.value] and type(o2) is type(o)}
    try:
        optimizer_provider.get("fedsgd")
        out["unknown_key"] = "no error"
    except ValueError as e:                 # object_factory.py:22-29
        out["unknown_key"] = "ValueError:" + str(e)

    # the job config's optimizer block {"sort": ..., "kwargs": ...} parsed by flame's own pydantic
    # model -- the class Config.optimizer is (config.py:121-123,209).  (The full Config(path) is not
    # parsed: the reference pins pydantic<2.0, lib/python/setup.py:43, and under this image's
    # pydantic 2 its Config requires fields transform_config never sets, e.g. `groups`.)
    from flame.config import Optimizer
    from diskcache import Cache
    blocks = {
        "fedyogi": {"sort": "fedyogi", "kwargs": {"beta_1": 0.85, "beta_2": 0.995, "eta": 0.02, "tau": 0.002}},
        "fedadam": {"sort": "fedadam", "kwargs": {"beta_1": 0.9, "beta_2": 0.99, "eta": 0.01, "tau": 0.001}},
        "fedbuff": {"sort": "fedbuff", "kwargs": {}},
        "fedavg_default": None,                    # no optimizer block: Optimizer() default (FEDAVG)
    }
    for name, blk in blocks.items():
        opt_cfg = Optimizer(**json.loads(json.dumps(blk))) if blk is not None else Optimizer()
        o = optimizer_provider.get(opt_cfg.sort, **opt_cfg.kwargs)
        out["config"][name] = {
            "sort": opt_cfg.sort.value, "cls": type(o).__module__ + "." + type(o).__name__,
            "hyper": [getattr(o, a, None) for a in ("beta_1", "beta_2", "eta", "tau")],
            "regularizer": type(o.regularizer).__module__,
        }
        # usable the way a role calls it with nothing received yet: do() on an empty cache
        # returns None without touching a GPU (fedavg.py:76-77, fedbuff.py:86-87)
        r = o.do(None, Cache(), total=0, version=1) if name == "fedbuff" else o.do({}, Cache(), total=0)
        out["config"][name]["empty_do"] = repr(r)
    try:
        Optimizer(sort="fednova", kwargs={})
        out["bad_sort"] = "accepted"
    except Exception as e:  # noqa: BLE001  (pydantic ValidationError: the closed enum, config.py:55-70)
        out["bad_sort"] = type(e).__name__
    print(json.dumps(out))


if __name__ == "__main__":
    main()
