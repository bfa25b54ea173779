"""FedAdam -- drop-in for lib/python/flame/optimizer/fedadam.py:25-35."""
from .fedopt import FedOPT


class FedAdam(FedOPT):
    """FedAdam class: v = beta_2*v + (1-beta_2)*d**2 (fedadam.py:33-35)."""

    variant = "fedadam"

    def __init__(self, beta_1=0.9, beta_2=0.99, eta=1e-2, tau=1e-3, defer: bool = False):
        super().__init__(beta_1, beta_2, eta, tau, defer=defer)

    def _delta_v_tensor(self, v, d):
        return self.beta_2 * v + (1 - self.beta_2) * d**2
