"""Child process of tests/test_env_classes.py: instantiates every drop-in the way flame's
roles do and prints, as JSON, which class each ``.regularizer`` (and FedGFT's server bias)
came from plus a few values computed with them.  Run with and without flame importable."""
import json
import sys

import torch

sys.path.insert(0, sys.argv[1])            # the repository root
from flame_amd.optimizers import optimizer_provider  # noqa: E402


class _LB:
    def __init__(self, a, b, c, d, val):
        self.a, self.b, self.c, self.d, self.val = a, b, c, d, val


def main():
    out = {}
    kw = {"fedavg": {}, "fedadam": {}, "fedyogi": {}, "fedadagrad": {}, "fedbuff": {}, "fedprox": {"mu": 0.01},
          "feddyn": {"alpha": 0.01}, "scaffold": {"k": 3}, "fedgft": {"fair": "SP", "gamma": 0.5}}
    for name, k in kw.items():
        opt = optimizer_provider.get(name, **k)
        r = opt.regularizer
        out[name] = {"module": type(r).__module__, "class": type(r).__name__}
    g = torch.Generator().manual_seed(3)
    w = [torch.randn(37, 5, generator=g), torch.randn(11, generator=g)]
    wt = [torch.randn(37, 5, generator=g), torch.randn(11, generator=g)]
    prox = optimizer_provider.get("fedprox", mu=0.01).regularizer
    out["fedprox_term"] = float(prox.get_term(w=w, w_t=wt))
    gft = optimizer_provider.get("fedgft", fair="SP", gamma=0.5)
    out["fedgft_bias_module"] = type(gft.bias).__module__
    sizes = {"e1": 300, "e2": 120, "e3": 77}
    gft.update_bias(dataset_sizes=sizes, local_biases={"e1": _LB(0.25, 0.5, 0.125, 0.75, 0.03125),
                                                        "e2": _LB(0.1, 0.2, 0.3, 0.4, -0.2),
                                                        "e3": _LB(0.7, 0.1, 0.9, 0.05, 0.5)})
    out["fedgft_bias"] = [gft.bias.a, gft.bias.b, gft.bias.c, gft.bias.d, gft.bias.val, gft.bias.sign]
    out["default_term"] = float(optimizer_provider.get("fedavg").regularizer.get_term(w=w, w_t=wt))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
