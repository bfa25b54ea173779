"""FedGFT -- drop-in for lib/python/flame/optimizer/fedgft.py:27-58.

On the server FedGFT IS FedAvg: the class inherits ``FedAvg.do`` unchanged
(fedgft.py:27) and adds only scalar bookkeeping of the group-fairness bias
that its top aggregator gathers from the trainers
(mode/horizontal/fedgft/top_aggregator.py:52-86):
``update_bias(dataset_sizes, local_biases)`` (fedgft.py:50-54) folds the
trainers' ``a, b, c, d`` (and ``val`` for SP/EOP) into sample-weighted means
(bias.py:63-103) and ``get_bias()`` returns ``val``.  The weighted reduction
is therefore the MI355X FedAvg kernel; the bias is host arithmetic on a
handful of Python floats.

When flame is importable its own ``Bias`` and ``FedGFTRegularizer`` are used
(trainers read ``.regularizer``, syncfl/trainer.py:74-77); otherwise the
restatements below.
"""
import logging

from .fedavg import FedAvg

logger = logging.getLogger(__name__)

_FAIR_KINDS = ("SP", "EOP", "CAL")


class _GroupBias:
    """Restatement of flame.optimizer.bias.Bias (bias.py:25-158).

    The group-fairness gap is ``a/b - c/d``.  A trainer-side (``local=True``)
    object measures ``a, b, c, d`` on its data and mirrors the global terms it
    receives; the server-side object (``local=False``) averages the trainers'
    terms weighted by dataset size.
    """

    def __init__(self, fair="", local=True):
        self.fair = fair
        self.a = self.b = self.c = self.d = 0.0
        self.val = 0.0
        self.sign = 0.0
        self.local = local
        if local:
            self.local_val = 0.0
            self.global_a = self.global_b = self.global_c = self.global_d = 1.0

    def update_bias(self, **kwargs):
        if self.local:                              # bias.py:64-72: copy the server's terms
            g = kwargs["global_bias"]
            self.global_a, self.global_b, self.global_c, self.global_d = g.a, g.b, g.c, g.d
            self.val, self.sign = g.val, g.sign
            return
        sizes, biases = kwargs["dataset_sizes"], kwargs["local_biases"]
        n = sum(sizes.values())

        def mean(attr):                             # bias.py:78-98, same term order and rounding
            return sum([getattr(biases[e], attr) * sizes[e] / n for e in biases])

        self.a, self.b, self.c, self.d = mean("a"), mean("b"), mean("c"), mean("d")
        if self.fair in ("SP", "EOP"):              # bias.py:100-106 (CAL keeps its val)
            self.val = mean("val")
        self.sign = 0.0 if self.val == 0 else (1.0 if self.val > 0 else -1.0)

    def calculate_bias_batch(self, output, target, group):
        """Per-batch terms (bias.py:110-131); ``output[:, 1]`` is the positive-class score."""
        import torch
        pos = output[:, 1]
        g0, g1 = group == 0, group == 1
        if self.fair == "SP":
            return torch.sum(pos * g0), torch.sum(g0), torch.sum(pos * g1), torch.sum(g1)
        if self.fair == "EOP":
            t0, t1 = g0 & (target == 1), g1 & (target == 1)
            return torch.sum(pos * t0), torch.sum(t0), torch.sum(pos * t1), torch.sum(t1)
        if self.fair == "CAL":
            t0, t1 = g0 & (target == 1), g1 & (target == 1)
            return torch.sum(pos * t0), torch.sum(pos * g0), torch.sum(pos * t1), torch.sum(pos * g1)
        raise ValueError("Fairness type not supported.")

    def calculate_bias(self, model, data_loader):
        import torch
        device = next(model.parameters()).device
        acc = torch.zeros(4)
        for data, target, group in data_loader:
            out = torch.exp(model(data.to(device)))
            acc += torch.Tensor(self.calculate_bias_batch(out, target.to(device), group.to(device)))
        return acc / len(data_loader.dataset)

    def update_local_bias_params(self, model, train_loader):
        import torch
        model.train(False)
        with torch.no_grad():
            a, b, c, d = self.calculate_bias(model, train_loader)
        self.a, self.c = a.item(), c.item()
        self.b, self.d = max(b.item(), 1e-8), max(d.item(), 1e-8)
        self.local_val = self.a / self.b - self.c / self.d
        self.val = self.a / self.global_b - self.c / self.global_d


try:  # pragma: no cover - depends on flame being installed
    from flame.optimizer.bias import Bias  # type: ignore
    from flame.optimizer.regularizer.fedgft import FedGFTRegularizer  # type: ignore
except Exception:  # noqa: BLE001
    from .regularizer import Regularizer

    Bias = _GroupBias

    class FedGFTRegularizer(Regularizer):
        """Restatement of optimizer/regularizer/fedgft.py:26-84 (trainer-side penalty)."""

        def __init__(self, fair, gamma, reg="l2"):
            super().__init__()
            self.fair, self.gamma, self.reg = fair, gamma, reg
            self.bias = Bias(fair=fair, local=True)

        def get_term(self, **kwargs):
            gamma = abs(self.bias.val * 2) if self.gamma == "auto" else self.gamma
            if self.fair:
                output, target, group = kwargs["output"], kwargs["target"], kwargs["group"]
                import torch
                a, _, c, _ = self.bias.calculate_bias_batch(torch.exp(output), target, group)
                gap = (a / self.bias.global_b - c / self.bias.global_d) / len(target)
                if self.fair == "CAL":
                    gap = -gap
                elif self.fair not in ("SP", "EOP"):
                    raise ValueError("Fairness type not supported")
            else:
                gap = 0.0
            coef = self.bias.sign if self.reg == "id" else self.bias.val
            return coef * gamma * gap

        def update_local_bias_params(self, model, train_loader):
            self.bias.update_local_bias_params(model, train_loader)

        def update_bias(self, global_bias):
            self.bias.update_bias(global_bias=global_bias)

        def get_local_bias(self):
            return self.bias.local_val


class FedGFT(FedAvg):
    """FedGFT class: FedAvg aggregation (HIP kernel) + server-side fairness bias."""

    def __init__(self, fair, gamma, reg="l2"):
        super().__init__()
        self.fair = fair
        self.regularizer = FedGFTRegularizer(fair, gamma, reg)
        self.bias = Bias(fair=self.fair, local=False)

    def update_bias(self, dataset_sizes, local_biases):
        self.bias.update_bias(dataset_sizes=dataset_sizes, local_biases=local_biases)
        logger.debug(f"current bias is {self.bias.val}")

    def get_bias(self):
        return self.bias.val
