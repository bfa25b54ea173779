"""FedYogi -- drop-in for lib/python/flame/optimizer/fedyogi.py:25-36."""
import torch

from .fedopt import FedOPT


class FedYogi(FedOPT):
    """FedYogi class: v = v - (1-beta_2)*d**2*sign(v - d**2) (fedyogi.py:34-36)."""

    variant = "fedyogi"

    def __init__(self, beta_1=0.9, beta_2=0.99, eta=1e-2, tau=1e-3, defer: bool = False):
        super().__init__(beta_1, beta_2, eta, tau, defer=defer)

    def _delta_v_tensor(self, v, d):
        return v - (1 - self.beta_2) * d**2 * torch.sign(v - d**2)
