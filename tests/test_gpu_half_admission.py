"""GPU: the 16-bit FedOPT steps' fast-path admission (adapt_vec_half, FLAME_T_HALF_ADMIT) over a
long eager run in which weights stop moving -- a client average that stays put lets the current
weight converge to it, d becomes exactly 0 and m decays by beta_1 per step, in bf16 down through
[2^-133, 2^-85], the range the fp32 step's admission sends to the general divide.  The bf16 step
now keeps those lanes on v_rcp_f32 (tools/fp_probe.py: equal under the bf16 rounding on every
bf16 numerator but NaN), fp16's m never gets there (its smallest nonzero value is 2^-24).

Every arrival's result, m_t and v_t are compared BITWISE with the reference's own op sequence
(OracleFedOPT: fedopt.py:58-129 as torch-CPU ops in the dtype, each op rounded to it), every
round, from the same starting weights -- not only within an ulp."""
import copy

import pytest
import torch

import scenarios as S

pytestmark = [pytest.mark.gpu, pytest.mark.oracle]

DEV = "cuda:0"


def _bitwise(label, got, exp):
    for k in exp:
        g, e = got[k].detach().cpu(), exp[k]
        assert g.dtype == e.dtype, (label, k, g.dtype, e.dtype)
        bad = (g.view(torch.int16) != e.view(torch.int16)).nonzero().flatten()
        assert bad.numel() == 0, (f"{label}/{k}: {bad.numel()} elements differ, first at {bad[:4].tolist()}: "
                                  f"{g[bad[:4]].tolist()} vs {e[bad[:4]].tolist()}")


@pytest.mark.parametrize("sort", ["fedadam", "fedyogi", "fedadagrad"])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16], ids=["bf16", "f16"])
def test_long_eager_run_with_stalled_weights_bitwise(sort, dtype):
    from oracle import oracle as O
    from flame_amd.optimizers import optimizer_provider
    n_el, arrivals, rounds = 2048 + 37, 32, 24
    g = torch.Generator().manual_seed(17)
    w0 = (torch.rand(n_el, generator=g) + 0.5).to(dtype)
    # round 1's clients move every weight; afterwards only the first half keeps receiving updates
    # (the rest average to exactly their base: d -> 0, m decays)
    def client(r, i):
        u = (torch.randn(n_el, generator=g) * 1e-2).to(dtype)
        if r > 0:
            u[n_el // 2:] = 0
        return u
    opt = optimizer_provider.get(sort, defer=True)
    ora = O.OracleFedOPT(sort)
    wa, wo = {"w": w0.to(DEV)}, {"w": w0.clone()}
    tiny_seen = 0
    for r in range(rounds):
        ba, bo = copy.deepcopy(wa), copy.deepcopy(wo)
        total = 0
        for i in range(arrivals):
            u, c = client(r, i), 1 + (i * 7) % 5
            total += c
            ca, co = S.SortedCache(), S.SortedCache()
            ca[f"r{r}e{i:03d}"] = S.TR({"w": u.to(DEV)}, c)
            co[f"r{r}e{i:03d}"] = S.TR({"w": u.clone()}, c)
            oa = opt.do(ba, ca, total=total)
            oo = ora.do(bo, co, total=total)
        wa, wo = {"w": dict(oa)["w"]}, oo
        _bitwise(f"{sort}/{dtype}/r{r}/base", S.to_cpu(ba), bo)
        _bitwise(f"{sort}/{dtype}/r{r}/current", S.to_cpu(wa), wo)
        if ora.m_t is not None:
            _bitwise(f"{sort}/{dtype}/r{r}/m", S.to_cpu(opt.m_t), ora.m_t)
            _bitwise(f"{sort}/{dtype}/r{r}/v", S.to_cpu(opt.v_t), ora.v_t)
            m = ora.m_t["w"].float().abs()
            tiny_seen += int(((m > 0) & (m < 2.0 ** -85)).sum())
    if dtype == torch.bfloat16:
        assert tiny_seen > 0          # the regime this test is for was reached (from round ~14)
