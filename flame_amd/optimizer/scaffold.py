"""SCAFFOLD -- drop-in for lib/python/flame/optimizer/scaffold.py:36-150.

Server side of SCAFFOLD (caller: mode/horizontal/scaffold/top_aggregator.py:71-126,
save_state at :160 and :177): ``do()`` first folds the trainers' control
variates into the global control ``c_glob`` in place with rate ``1/n_clnt``
(``n_clnt = len(weight_dict)``, :116-122, ``c_aggregate_fn`` :141-150), then
is FedAvg over the model updates with the uniform rate ``1/len(cache)``
(:127-134).  Both are the sequential weighted client reduction: one
``flame_agg_reduce`` launch per dtype over every key and every trainer,
bit-identical to the reference's per-trainer / per-key torch-CPU loop.
A control variate whose dtype differs from ``c_glob``'s runs the reference's
statements (``(v*rate).to(c.dtype)`` then ``+=``) as ``flame_elementwise`` programs.

``c_glob`` is created ``zeros_like`` the global weights (:81-90), but in HBM:
it is state the server updates every round and only reads out when it sends
it to trainers (``weights_to_device(c_glob, CPU)``, top_aggregator.py:193).
"""
import logging

import torch

from .. import elementwise as ew, engine
from .fedavg import FedAvg

logger = logging.getLogger(__name__)

DATASET_SIZES = "dataset_sizes"
GLOBAL_WEIGHTS = "glob_weights"

try:  # pragma: no cover - depends on flame being installed
    from flame.optimizer.regularizer.scaffold import ScaffoldRegularizer  # type: ignore
except Exception:  # noqa: BLE001
    ScaffoldRegularizer = None


def _is_pre(state) -> bool:
    return getattr(state, "value", state) == "pre"   # flame.common.constants.TrainState.PRE


class Scaffold(FedAvg):
    """SCAFFOLD class."""

    def __init__(self, k):
        super().__init__()
        self.c_glob = None
        if ScaffoldRegularizer is not None:
            self.regularizer = ScaffoldRegularizer(k)

    def save_state(self, state, **kwargs):
        """scaffold.py:58-90: client weights from dataset sizes; zero c_glob on first weights."""
        if not _is_pre(state):
            return
        if DATASET_SIZES in kwargs:
            dataset_sizes = kwargs[DATASET_SIZES]
            total_samples = sum(dataset_sizes.values())
            num_trainers = len(dataset_sizes)
            self.weight_dict = {end: (dataset_sizes[end] / total_samples) * num_trainers
                                for end in dataset_sizes}
        if GLOBAL_WEIGHTS in kwargs and self.c_glob is None:
            glob = kwargs[GLOBAL_WEIGHTS]
            device = engine.pick_device(glob)
            self.c_glob = {k: torch.zeros(glob[k].shape, dtype=glob[k].dtype, device=device) for k in glob}

    def do(self, base_weights, cache, *, total: int = 0, version: int = 0, **kwargs):
        logger.debug("calling scaffold (flame_amd)")
        assert base_weights is not None
        if len(cache) == 0 or total == 0:
            return None
        control_cache = kwargs["control_cache"]
        if len(control_cache) != len(cache):
            return None

        self.c_agg_weights = self.c_glob
        rate = 1 / len(self.weight_dict)
        controls = [control_cache.pop(k).weights for k in list(control_cache.iterkeys())]
        self._c_aggregate(controls, rate)
        self.c_glob = self.c_agg_weights

        self.agg_weights = base_weights
        rate = 1 / len(cache)
        entries = [(cache.pop(k).weights, rate) for k in list(cache.iterkeys())]
        engine.accumulate(self.agg_weights, entries)
        return self.agg_weights

    def _c_aggregate(self, controls, rate):
        """c[k] += (v*rate) cast to c[k].dtype, trainer by trainer (scaffold.py:141-150)."""
        if not controls:
            return
        c = self.c_agg_weights
        device = engine.pick_device(c, *controls)
        same = [k for k in c if all(k in w for w in controls) and all(w[k].dtype == c[k].dtype for w in controls)]
        if same:
            engine.accumulate({k: c[k] for k in same}, [({k: w[k] for k in same}, rate) for w in controls],
                              device=device)
        for w in controls:   # keys with another dtype, in trainer order: the reference's statements
            for k in w.keys():   # as flame_elementwise programs (elementwise.py)
                if k in same:
                    continue
                tmp = ew.Lazy.of(engine.logical_tensor(w, k)) * rate
                ew.iadd(c[k], tmp.to(c[k].dtype) if tmp.dtype != c[k].dtype else tmp)
