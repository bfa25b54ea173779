"""GPU: the fp16 eager FedOPT chain on packed halves (fedopt_chain_body_f16, FLAME_T_F16_NATIVE)
against the reference's own op sequence (OracleFedOPT: fedopt.py:58-129 as torch-CPU ops in fp16,
each op rounded to fp16), BITWISE, on values chosen to reach the corners of the packed step:
subnormal and near-overflow updates, signed zeros, weights that stop moving, and a model whose
full 2048-element chunks (the packed path) sit beside a ragged tail chunk (the per-element path).

Corners the packed step argues for (fedagg.hip): an fp16 op on two fp16 operands rounded once
equals torch's fp32 op rounded to fp16 (Figueroa), the scalar products through v_fma_mix_f32 keep
signed zeros, FedYogi's sign of a pair keeps +0 for -0.  A non-finite case checks that a lane
whose v overflows takes the general path and matches the reference up to NaN payloads."""
import copy

import pytest
import torch

import scenarios as S

pytestmark = [pytest.mark.gpu, pytest.mark.oracle]

DEV = "cuda:0"
SORTS = ["fedadam", "fedyogi", "fedadagrad"]


def _same(label, got, exp, nan_ok=False):
    for k in exp:
        g, e = got[k].detach().cpu(), exp[k]
        assert g.dtype == e.dtype == torch.float16, (label, k, g.dtype, e.dtype)
        gb, eb = g.view(torch.int16), e.view(torch.int16)
        diff = gb != eb
        if nan_ok:                      # NaN payloads are not part of the contract
            diff &= ~(torch.isnan(g) & torch.isnan(e))
        bad = diff.nonzero().flatten()
        assert bad.numel() == 0, (f"{label}/{k}: {bad.numel()} elements differ, first at {bad[:4].tolist()}: "
                                  f"{g[bad[:4]].tolist()} vs {e[bad[:4]].tolist()}")


def _edge_update(g, n, r, scale_pow):
    """A client update mixing magnitudes 2^-30 .. 2^scale_pow (fp16 subnormals included), exact
    zeros of both signs, and weights that receive nothing after round 0."""
    u = torch.randn(n, generator=g) * torch.pow(2.0, torch.randint(-30, scale_pow + 1, (n,), generator=g).float())
    z = torch.rand(n, generator=g)
    u[z < 0.05] = 0.0
    u[(z >= 0.05) & (z < 0.10)] = -0.0
    u[n // 2:n // 2 + 64] = -0.0    # a block of -0 weights that only ever receives -0: b stays -0
    if r > 0:
        u[n - n // 4:] = 0.0        # stalled weights: d -> 0, m decays through the fp16 subnormals
    return u.to(torch.float16)


def _run(sort, n_el, rounds, arrivals, scale_pow, seed, beta_1=0.9, beta_2=0.99, eta=1e-2, tau=1e-3,
         nan_ok=False, w0=None):
    from oracle import oracle as O
    from flame_amd.optimizers import optimizer_provider
    g = torch.Generator().manual_seed(seed)
    if w0 is None:
        w0 = (torch.randn(n_el, generator=g) * 4).to(torch.float16)
        w0[:64] = torch.tensor([0.0, -0.0, 6.0e-8, -6.0e-8, 65504.0, -65504.0, 1.0e-4, -1.0e-4] * 8,
                               dtype=torch.float16)
        w0[n_el // 2:n_el // 2 + 64] = -0.0
    opt = optimizer_provider.get(sort, beta_1=beta_1, beta_2=beta_2, eta=eta, tau=tau, defer=True)
    ora = O.OracleFedOPT(sort, beta_1=beta_1, beta_2=beta_2, eta=eta, tau=tau)
    wa, wo = {"w": w0.to(DEV)}, {"w": w0.clone()}
    for r in range(rounds):
        ba, bo = copy.deepcopy(wa), copy.deepcopy(wo)
        total = 0
        for i in range(arrivals):
            u, c = _edge_update(g, n_el, r, scale_pow), 1 + (i * 5) % 7
            total += c
            ca, co = S.SortedCache(), S.SortedCache()
            ca[f"r{r}e{i:03d}"] = S.TR({"w": u.to(DEV)}, c)
            co[f"r{r}e{i:03d}"] = S.TR({"w": u.clone()}, c)
            oa = opt.do(ba, ca, total=total)
            oo = ora.do(bo, co, total=total)
        wa, wo = {"w": dict(oa)["w"]}, oo
        _same(f"{sort}/r{r}/base", S.to_cpu(ba), bo, nan_ok)
        _same(f"{sort}/r{r}/current", S.to_cpu(wa), wo, nan_ok)
        if ora.m_t is not None:
            _same(f"{sort}/r{r}/m", S.to_cpu(opt.m_t), ora.m_t, nan_ok)
            _same(f"{sort}/r{r}/v", S.to_cpu(opt.v_t), ora.v_t, nan_ok)
    return opt, ora


@pytest.mark.parametrize("sort", SORTS)
def test_f16_chain_edge_values_bitwise(sort):
    # 3 full chunks of 2048 (the packed path) + a 301-element tail chunk (the per-element path)
    _run(sort, 3 * 2048 + 301, rounds=6, arrivals=12, scale_pow=4, seed=101, nan_ok=True)   # +-65504 weights overflow


@pytest.mark.parametrize("sort", SORTS)
def test_f16_chain_large_updates_bitwise(sort):
    # updates up to 2^12: d^2 overflows fp16 for some weights (v = inf: the general path)
    _run(sort, 2 * 2048 + 7, rounds=3, arrivals=8, scale_pow=12, seed=202, nan_ok=True)


@pytest.mark.parametrize("sort", SORTS)
def test_f16_chain_other_hyperparameters_bitwise(sort):
    # eta > 1 (numerators near overflow), a large tau (den near its fp16 bound) and a beta_2 > 1
    # (FedYogi's t <= 0, FedAdam's (1 - beta_2) < 0)
    _run(sort, 2048 + 129, rounds=4, arrivals=9, scale_pow=2, seed=303, beta_1=0.5, beta_2=1.25, eta=4.0,
         tau=1024.0, nan_ok=True)
