"""FedAdaGrad -- drop-in for lib/python/flame/optimizer/fedadagrad.py:25-35."""
from .fedopt import FedOPT


class FedAdaGrad(FedOPT):
    """FedAdaGrad class: v = v + d**2 (fedadagrad.py:33-35)."""

    variant = "fedadagrad"

    def __init__(self, beta_1=0.9, beta_2=0.99, eta=1e-2, tau=1e-3, defer: bool = False):
        super().__init__(beta_1, beta_2, eta, tau, defer=defer)

    def _delta_v_tensor(self, v, d):
        return v + d**2
