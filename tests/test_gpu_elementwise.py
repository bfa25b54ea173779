"""GPU: the keys the fused FedOPT kernel does not take -- an int64 0-dim num_batches_tracked, int32 /
uint8 / int16 buffers, fp64 tensors, bf16 / fp16 keys whose current weights were promoted, and the
keys that come out of those promotions in later rounds -- run as flame_elementwise programs
(flame_amd/elementwise.py), against the reference's torch op sequence (OracleFedOPT._adapt_torch:
fedopt.py:102-129 + the variant's _delta_v, torch-CPU), several syncfl rounds, every key of
current_weights, m_t and v_t:
  * BITWISE against the op sequence with the fp32 root correctly rounded (``sqrt_rn``: what the
    kernels compute, torch-CPU's own fp32 sqrt being ~1 ulp off on ~0.6 % of values);
  * within SURVEY §8(c)'s fp32 contract against plain torch-CPU.
Each round starts both from the GPU's state (weights, m_t, v_t), as test_chain_vs_oracle does."""
import copy

import pytest
import torch

import scenarios as S

pytestmark = [pytest.mark.gpu, pytest.mark.oracle]

DEV = "cuda:0"
SORTS = ["fedadam", "fedyogi", "fedadagrad"]

# key -> (dtype, shape, value scale): the fused kernel takes only "w"
# (keys of one dtype / 0-dim signature share one program and ONE flame_elementwise_segments launch:
# the two num_batches_tracked, the two int32 buffers of different lengths)
KEYS = {"w": (torch.float32, (300,), 1.0), "num_batches_tracked": (torch.int64, (), 0),
        "cnt": (torch.int32, (7,), 0), "d64": (torch.float64, (513,), 1.0), "u8": (torch.uint8, (33,), 0),
        "i16": (torch.int16, (9,), 0), "h": (torch.bfloat16, (64,), 1.0),
        "bn2.num_batches_tracked": (torch.int64, (), 0), "cnt2": (torch.int32, (1031,), 0)}


def _tensor(g, dt, shape, scale, r, i):
    if dt.is_floating_point:
        return (torch.randn(shape, generator=g, dtype=torch.float64) * scale).to(dt)
    hi = 200 if dt == torch.uint8 else 1000
    return torch.randint(0, hi, shape, generator=g).to(dt) + (r * 10 + i if dt != torch.uint8 else 0)


def _same(label, got, exp):
    for k in exp:
        g, e = got[k].detach().cpu(), exp[k]
        assert g.dtype == e.dtype and g.shape == e.shape, (label, k, g.dtype, e.dtype, g.shape, e.shape)
        if g.dtype.is_floating_point:
            both_nan = torch.isnan(g) & torch.isnan(e)
            bad = ((g.view(-1) != e.view(-1)) | (torch.signbit(g.view(-1)) != torch.signbit(e.view(-1)))) & ~both_nan.view(-1)
        else:
            bad = g.view(-1) != e.view(-1)
        idx = bad.nonzero().flatten()
        assert idx.numel() == 0, (f"{label}/{k} ({g.dtype}): {idx.numel()} of {g.numel()} differ, first at "
                                  f"{idx[:4].tolist()}: {g.view(-1)[idx[:4]].tolist()} vs {e.view(-1)[idx[:4]].tolist()}")


@pytest.mark.parametrize("sort", SORTS)
def test_fedopt_keys_outside_the_fused_kernel_vs_oracle(sort):
    from oracle import oracle as O
    from flame_amd import engine
    from flame_amd.optimizers import optimizer_provider
    g = torch.Generator().manual_seed(61 + SORTS.index(sort))
    weights = {k: _tensor(g, dt, sh, sc, 0, 0) for k, (dt, sh, sc) in KEYS.items()}
    opt = optimizer_provider.get(sort)
    launches = []
    engine._recorders.append(launches)
    try:
        for r in range(4):
            n = 5
            ups = [{k: _tensor(g, dt, sh, sc * 0.1, r + 1, i) for k, (dt, sh, sc) in KEYS.items()} for i in range(n)]
            counts = [int(c) for c in torch.randint(1, 50, (n,), generator=g)]
            oras = {"rn": O.OracleFedOPT(sort, sqrt_rn=True), "torch": O.OracleFedOPT(sort)}
            outs = {}
            for name, ora in oras.items():       # each from the GPU's state at the round's start
                if r > 0:
                    ora.current_weights = S.to_cpu(opt.current_weights)
                    if opt.m_t is not None:
                        ora.m_t, ora.v_t = S.to_cpu(opt.m_t), S.to_cpu(opt.v_t)
                cache, total = S.SortedCache(), 0
                for i, (u, c) in enumerate(zip(ups, counts)):
                    total += c
                    cache[f"r{r}e{i}"] = S.TR({k: t.clone() for k, t in u.items()}, c)
                outs[name] = ora.do(copy.deepcopy(S.to_cpu(weights)), cache, total=total)
            cache, total = S.SortedCache(), 0
            for i, (u, c) in enumerate(zip(ups, counts)):
                total += c
                cache[f"r{r}e{i}"] = S.TR(S.to_dev(u, DEV), c)
            got = opt.do(copy.deepcopy(S.to_dev(weights, DEV)), cache, total=total)
            weights = S.to_cpu(got)
            _same(f"{sort}/r{r}/current", got, outs["rn"])
            # (a key whose reference result holds NaNs -- int16's d ** 2 wraps negative, its root is
            # NaN -- is held by the bitwise check above only)
            fin = [k for k, t in outs["torch"].items() if not t.is_floating_point() or bool(torch.isfinite(t).all())]
            S.assert_close_fedopt(f"{sort}/r{r}/current vs torch-CPU", {k: got[k] for k in fin},
                                  {k: outs["torch"][k] for k in fin})
            if oras["rn"].m_t is not None:
                _same(f"{sort}/r{r}/m", opt.m_t, oras["rn"].m_t)
                _same(f"{sort}/r{r}/v", opt.v_t, oras["rn"].v_t)
    finally:
        engine._recorders.remove(launches)
    names = [ev[0] for ev in launches]
    assert "flame_elementwise" in names and "flame_elementwise_segments" in names, names
    # the promoted keys end the run in fp32 (int * python float -> fp32), AdaGrad's int v aside
    assert got["num_batches_tracked"].dtype == torch.float32 and got["d64"].dtype == torch.float64


@pytest.mark.parametrize("sort", SORTS)
def test_fedopt_int_and_fp64_keys_edge_values(sort):
    """Edge values through the elementwise program: int64 near 2^62 (d**2 wraps in int64), uint8
    wrap-around (3 - 5 = 254), fp64 zeros of both signs, subnormals, huge values."""
    from oracle import oracle as O
    from flame_amd.optimizers import optimizer_provider
    base = {"i": torch.tensor([2 ** 62, -(2 ** 62), 3, 0, -7, 2 ** 31 + 5], dtype=torch.int64),
            "u": torch.tensor([3, 5, 250, 0, 255, 1], dtype=torch.uint8),
            "f": torch.tensor([0.0, -0.0, 5e-324, -1e308, 1e-300, 3.5], dtype=torch.float64)}
    ups = [{"i": torch.tensor([5, -3, 2 ** 40, 1, 0, -2 ** 33], dtype=torch.int64),
            "u": torch.tensor([5, 3, 10, 255, 0, 2], dtype=torch.uint8),
            "f": torch.tensor([-0.0, 0.0, 1e-310, 1e308, -1e-300, 2.0], dtype=torch.float64)},
           {"i": torch.tensor([-1, 2 ** 61, 7, -9, 4, 3], dtype=torch.int64),
            "u": torch.tensor([1, 200, 4, 9, 17, 250], dtype=torch.uint8),
            "f": torch.tensor([1.0, -2.0, 0.0, -0.0, 7.0, 1e-320], dtype=torch.float64)}]
    opt = optimizer_provider.get(sort)
    ora = O.OracleFedOPT(sort, sqrt_rn=True)
    wg, wo = S.to_dev(base, DEV), {k: v.clone() for k, v in base.items()}
    for r in range(3):
        cg, co, total = S.SortedCache(), S.SortedCache(), 0
        for i, u in enumerate(ups):
            total += 3 + i
            cg[f"r{r}e{i}"] = S.TR(S.to_dev(u, DEV), 3 + i)
            co[f"r{r}e{i}"] = S.TR({k: v.clone() for k, v in u.items()}, 3 + i)
        wg = opt.do(copy.deepcopy(wg), cg, total=total)
        wo = ora.do(copy.deepcopy(wo), co, total=total)
        _same(f"{sort}/r{r}/current", wg, wo)
        if ora.m_t is not None:
            _same(f"{sort}/r{r}/m", opt.m_t, ora.m_t)
            _same(f"{sort}/r{r}/v", opt.v_t, ora.v_t)
