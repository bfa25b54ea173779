"""FedProx -- drop-in for lib/python/flame/optimizer/fedprox.py:28-46.

On the server FedProx IS FedAvg (the proximal term lives in the trainers'
loss), so ``do()`` is the MI355X FedAvg kernel.  Trainers instantiate the
optimizer to read ``.regularizer`` (syncfl/trainer.py:74-77): flame's own
FedProxRegularizer is used when flame is importable, otherwise an equivalent
restatement of optimizer/regularizer/fedprox.py:24-47.
"""
from .fedavg import FedAvg

try:  # pragma: no cover - depends on flame being installed
    from flame.optimizer.regularizer.fedprox import FedProxRegularizer  # type: ignore
except Exception:  # noqa: BLE001
    from .regularizer import Regularizer

    class FedProxRegularizer(Regularizer):
        """(mu/2) * ||w - w_t||^2 over the concatenated parameters."""

        def __init__(self, mu):
            super().__init__()
            self.mu = mu
            self.state_dict = dict()

        @staticmethod
        def _vec(params):
            import torch
            return torch.cat([p.reshape(-1) for p in params])

        def get_term(self, **kwargs):
            import torch
            w_vector = self._vec(kwargs["w"])
            if "w_t_vector" not in self.state_dict:
                self.state_dict["w_t_vector"] = self._vec(kwargs["w_t"])
            return (self.mu / 2) * torch.sum(torch.pow(w_vector - self.state_dict["w_t_vector"], 2))

        def update(self):
            del self.state_dict["w_t_vector"]


class FedProx(FedAvg):
    """FedProx class (server side = FedAvg)."""

    def __init__(self, mu):
        super().__init__()
        self.mu = mu
        self.regularizer = FedProxRegularizer(self.mu)
