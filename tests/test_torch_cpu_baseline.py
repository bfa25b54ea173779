"""The CPU baseline bench.py times (oracle/torch_cpu.py) is the reference's own op
sequence: replayed through the golden drivers it reproduces the reference's
outputs bitwise -- FedOPT included, since it is the same torch-CPU sqrt."""
import pytest
import torch

import scenarios as S
from oracle import torch_cpu


class _FedAvg:
    def __init__(self):
        self.agg_weights = None

    def do(self, base_weights, cache, *, total=0, version=0, **kwargs):
        self.agg_weights = base_weights
        if len(cache) == 0 or total == 0:
            return None
        for k in list(cache.iterkeys()):
            tres = cache.pop(k)
            torch_cpu.fedavg_round(self.agg_weights, [tres.weights], [tres.count], total)
        return self.agg_weights


class _FedOPT(_FedAvg):
    def __init__(self, sort, beta_1, beta_2, eta, tau):
        super().__init__()
        self.sort, self.hyper = sort, (beta_1, beta_2, eta, tau)
        self.current_weights, self.m_t, self.v_t = None, None, None

    def do(self, base_weights, cache, *, total=0, version=0, **kwargs):
        avg = super().do(base_weights, cache, total=total)
        if avg is None:
            return self.current_weights
        if self.current_weights is None:
            self.current_weights = avg
            return avg
        if self.m_t is None:
            self.m_t, self.v_t = {}, {}
        self.current_weights = torch_cpu.fedopt_adapt(self.sort, avg, self.current_weights, self.m_t, self.v_t,
                                                      *self.hyper)
        return self.current_weights


class _FedBuff:
    def do(self, agg, cache, *, total=0, version=0, **kwargs):
        if len(cache) == 0 or total == 0:
            return None
        start_none = agg is None
        for k in list(cache.iterkeys()):
            tres = cache.pop(k)
            agg = torch_cpu.fedbuff_step(None if start_none else agg, tres.weights, version, tres.version)
        return agg

    def scale_add_agg_weights(self, base, agg, goal):
        return torch_cpu.fedbuff_scale_add(base, agg, goal)


def _make(sort, **kw):
    return {"fedavg": _FedAvg, "fedbuff": _FedBuff}[sort]() if sort in ("fedavg", "fedbuff") else _FedOPT(sort, **kw)


@pytest.mark.parametrize("name,driver", [
    ("fedavg_small.npz", S.run_fedavg), ("fedavg_dtypes.npz", S.run_fedavg), ("fedavg_eager.npz", S.run_fedavg_eager),
    ("fedbuff_seq_fp32.npz", S.run_fedbuff_seq), ("fedbuff_seq_bf16.npz", S.run_fedbuff_seq),
    ("fedadam_rounds.npz", S.run_fedopt), ("fedyogi_rounds.npz", S.run_fedopt),
    ("fedadagrad_rounds.npz", S.run_fedopt), ("fedadam_mixed_rounds.npz", S.run_fedopt)])
def test_torch_cpu_matches_golden(golden, name, driver):
    for label, got, exp in driver(golden(name), _make, "cpu"):
        S.assert_bitwise(f"{name}:{label}", got, exp)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16, torch.float64])
def test_oracle_nonfinite_matches_reference_ops(dtype):
    """NaN / inf / overflowing client updates: the C oracle puts NaN and +-inf exactly where
    the reference's torch-CPU op sequence (fedavg.py:84-104) does."""
    from oracle import oracle as O
    base, cl, counts = S.nonfinite_case(dtype)
    tot = sum(counts)
    exp = {"w": base.clone()}
    torch_cpu.fedavg_round(exp, [{"w": c} for c in cl], counts, tot)
    got = base.clone()
    O.reduce_tensor(got, cl, [c / tot for c in counts])
    assert torch.isinf(exp["w"]).sum() > 10 and torch.isnan(exp["w"]).sum() > 10
    S.assert_same_nonfinite(str(dtype), got, exp["w"])
