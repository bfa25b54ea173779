"""GPU: the FedOPT step's fast correctly rounded sqrt / divide (flame_amd/csrc/fastmath.h) and its
per-lane fallback (adapt_vec), against the C oracle, bit for bit.

adapt_vec takes sqrt_rn / div_rn for a lane only when each of its elements' v is in [+0, 2^78]
and each eta*m is +-0 or in [2^-85, 2^100]; any other operand sends that lane through the general
sequences (the rest of its wave stays on the fast path).  On [2^-96, 2^78] both are correctly
rounded, as the C oracle's sqrtf and division are (oracle/fedagg_oracle.c:191-220,
fedopt.py:102-129); below 2^-96 sqrt_rn is not, but sqrt(v) + tau is tau either way
(fastmath.h).  So fp32 results equal the oracle's bitwise -- on either side of every admission
boundary.  A tiny eta (1e-25) puts every eta*m below 2^-85: all lanes on the general divide.
The model below puts one boundary case in each of a run of waves (a wave = 64 lanes x 4 fp32
elements), the rest of them ordinary, and runs the per-call fused kernel (three rounds:
passthrough, zero state, running state) and the deferred eager chain against OracleFedOPT.  NaN / inf positions are checked separately (their payloads
are not part of the contract).
"""
import copy

import pytest
import torch

import scenarios as S

pytestmark = [pytest.mark.gpu, pytest.mark.oracle]

DEV = "cuda:0"
SORTS = ["fedadam", "fedyogi", "fedadagrad"]
ETAS = [None, 1e-25]    # None: the optimizer's default; 1e-25: every eta*m below 2^-85
WAVE = 256          # fp32 elements per wave of the FedOPT kernels (64 lanes x 4)

# One element per case: its current weight is 0 and every client sends the same value d, so the
# round's average is 0 + sum(rate_i * d) ~ d and the step's d, v, eta*m land on the named side of
# a boundary (fedopt.py:106-129; Adam / Yogi v = 0.01 d^2 from zero state, AdaGrad v = d^2).
CASES = [
    ("ordinary", None),
    ("zero d", 0.0),                    # v = +0 and eta*m = +0: admitted
    ("v below 2^-96", 1e-15),           # v ~ 1e-32 (AdaGrad 1e-30)
    ("v subnormal", 1e-22),             # AdaGrad: d^2 ~ 1e-44
    ("v above 2^78", 1e18),             # v ~ 1e34
    ("v inf", 3e20),                    # d^2 overflows
    ("eta*m below 2^-85", 1e-24),       # v underflows to 0, eta*m ~ 1e-27
    ("eta*m tiny negative", -1e-24),
    ("v just above 2^-96", 4e-14),      # Adam / Yogi: 1.6e-29
    ("v just below 2^-96", 3e-14),      # Adam / Yogi: 9.0e-30
    ("nan", float("nan")),
    ("large negative d", -1e13),        # v ~ 1e24 (AdaGrad 1e26)
]


def _case_elem(i):
    return i * WAVE + (13 * i) % WAVE


def _model(n_waves_ordinary=5):
    """One key: a wave per case (one lane's element carrying it, at a varying lane, the rest
    ordinary), then ordinary waves and a ragged tail."""
    g = torch.Generator().manual_seed(71)
    n = (len(CASES) + n_waves_ordinary) * WAVE + 37
    cur = torch.rand(n, generator=g) * 0.5 + 0.25
    for i, (_, d) in enumerate(CASES):
        if d is not None:
            cur[_case_elem(i)] = 0.0
    return cur


def _updates(n_el, n, g):
    ups = [torch.randn(n_el, generator=g) * 1e-2 for _ in range(n)]
    for i, (_, d) in enumerate(CASES):
        if d is not None:
            for u in ups:
                u[_case_elem(i)] = d
    return ups


def _bits_equal_or_both_nan(label, got, exp):
    for k in exp:
        gt, et = got[k].detach().cpu(), exp[k]
        nan = torch.isnan(et)
        assert torch.equal(torch.isnan(gt), nan), f"{label}/{k}: NaN positions differ"
        keep = ~nan
        bad = (gt[keep].view(torch.int32) != et[keep].view(torch.int32)).nonzero().flatten()
        assert bad.numel() == 0, (f"{label}/{k}: {bad.numel()} elements differ from the oracle, first at "
                                  f"{keep.nonzero().flatten()[bad[:4]].tolist()}: {gt[keep][bad[:4]].tolist()} vs "
                                  f"{et[keep][bad[:4]].tolist()}")


def _kw(eta):
    return {} if eta is None else {"eta": eta}


@pytest.mark.parametrize("eta", ETAS)
@pytest.mark.parametrize("sort", SORTS)
def test_fused_step_admission_boundaries_bitwise(sort, eta):
    from oracle import oracle as O
    from flame_amd.optimizers import optimizer_provider
    cur = _model()
    g = torch.Generator().manual_seed(5)
    amd, ora = optimizer_provider.get(sort, **_kw(eta)), O.OracleFedOPT(sort, **_kw(eta))
    wa, wo = {"w": cur.to(DEV)}, {"w": cur.clone()}
    for r in range(3):
        ups = _updates(cur.numel(), 4, g)
        counts = [3, 5, 7, 11]
        ca, co = S.SortedCache(), S.SortedCache()
        for i, u in enumerate(ups):
            ca[f"{i}"] = S.TR({"w": u.to(DEV)}, counts[i])
            co[f"{i}"] = S.TR({"w": u.clone()}, counts[i])
        wa = amd.do({"w": wa["w"].clone()}, ca, total=sum(counts))
        wo = ora.do({"w": wo["w"].clone()}, co, total=sum(counts))
        _bits_equal_or_both_nan(f"{sort}/r{r}/avg", S.to_cpu(amd.agg_weights), ora.agg_weights)
        _bits_equal_or_both_nan(f"{sort}/r{r}/cur", S.to_cpu(wa), wo)
        if r >= 1:
            _bits_equal_or_both_nan(f"{sort}/r{r}/m", S.to_cpu(amd.m_t), ora.m_t)
            _bits_equal_or_both_nan(f"{sort}/r{r}/v", S.to_cpu(amd.v_t), ora.v_t)


@pytest.mark.parametrize("eta", ETAS)
@pytest.mark.parametrize("sort", SORTS)
def test_chain_admission_boundaries_bitwise(sort, eta):
    """The eager round through FedOPT(defer=True) (one flame_fedopt_chain launch per round): 6
    arrivals per round, two rounds, every returned current, m_t and v_t == the oracle's
    per-call sequence, bitwise."""
    from oracle import oracle as O
    from flame_amd.optimizers import optimizer_provider
    cur = _model()
    g = torch.Generator().manual_seed(9)
    rounds = [[(u, 2 + 3 * i) for i, u in enumerate(_updates(cur.numel(), 6, g))] for _ in range(2)]
    opt, ora = optimizer_provider.get(sort, defer=True, **_kw(eta)), O.OracleFedOPT(sort, **_kw(eta))
    wa, wo = {"w": cur.to(DEV)}, {"w": cur.clone()}
    for r, arrivals in enumerate(rounds):
        ba, bo = copy.deepcopy(wa), copy.deepcopy(wo)
        ca, co = S.SortedCache(), S.SortedCache()
        total = 0
        for i, (u, c) in enumerate(arrivals):
            total += c
            ca[f"r{r}e{i}"] = S.TR({"w": u.to(DEV)}, c)
            co[f"r{r}e{i}"] = S.TR({"w": u.clone()}, c)
            oa = opt.do(ba, ca, total=total)
            oo = ora.do(bo, co, total=total)
        wa, wo = S.to_cpu(dict(oa)), oo
        wa = {"w": wa["w"].to(DEV)}
        _bits_equal_or_both_nan(f"chain/{sort}/r{r}/base", S.to_cpu(ba), bo)
        _bits_equal_or_both_nan(f"chain/{sort}/r{r}/cur", S.to_cpu(wa), wo)
        _bits_equal_or_both_nan(f"chain/{sort}/r{r}/m", S.to_cpu(opt.m_t), ora.m_t)
        _bits_equal_or_both_nan(f"chain/{sort}/r{r}/v", S.to_cpu(opt.v_t), ora.v_t)

