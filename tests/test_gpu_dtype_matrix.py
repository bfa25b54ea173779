"""GPU: the FedAvg / FedBuff drop-ins against torch CPU itself (the reference's arithmetic,
fedavg.py:93-104, fedbuff.py:122-157) for every pair of (aggregate dtype, update dtype) a
state_dict can carry -- bitwise, errors included -- with several arrivals per key (the
kernel's in-order sum) and a FedBuff scale_add into a model of each float dtype."""
import math

import pytest
import torch

import scenarios as S
from oracle import torch_cpu
from test_oracle_dtype_matrix import DTYPES, _rand, _reference

pytestmark = [pytest.mark.gpu, pytest.mark.oracle]

DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _native_loaded():
    from flame_amd import _native
    _native.lib()
    assert torch.cuda.is_available()


def _drop_in(sort):
    from flame_amd.optimizers import optimizer_provider
    return optimizer_provider.get(sort)


@pytest.mark.parametrize("acc_dt", DTYPES, ids=[str(d)[6:] for d in DTYPES])
def test_fedavg_every_dtype_pair_vs_torch(acc_dt):
    g = torch.Generator().manual_seed(7 + DTYPES.index(acc_dt))
    for v_dt in DTYPES:
        acc = _rand(g, acc_dt, 4099, 1.0)
        vs = [_rand(g, v_dt, 4099, 1e-1) for _ in range(3)]
        counts = [5, 11, 17]
        exp = acc.clone()
        try:
            for v, c in zip(vs, counts):
                _reference(exp, v, c / sum(counts))
            err = None
        except RuntimeError as e:
            err = e
        cache = S.SortedCache()
        for i, (v, c) in enumerate(zip(vs, counts)):
            cache[f"e{i}"] = S.TR({"k": v.to(DEV)}, c)
        base = {"k": acc.to(DEV)}
        if err is not None:
            with pytest.raises(RuntimeError):
                _drop_in("fedavg").do(base, cache, total=sum(counts))
            continue
        out = _drop_in("fedavg").do(base, cache, total=sum(counts))
        S.assert_bitwise(f"{acc_dt}+={v_dt}", {"k": out["k"]}, {"k": exp})


@pytest.mark.parametrize("agg_dt", [torch.float32, torch.bfloat16, torch.float16, torch.float64, torch.int64,
                                    torch.uint8])
def test_fedbuff_scale_add_every_model_dtype_vs_torch(agg_dt):
    """FedBuff None start in agg_dt, then scale_add into a model of every float dtype
    (``base += agg / goal``: the quotient in agg's dtype -- float32 for integers -- then
    the promoted add)."""
    g = torch.Generator().manual_seed(40 + int(agg_dt.itemsize))
    ups = [_rand(g, agg_dt, 2051, 1e-1) for _ in range(3)]
    for model_dt in (torch.float32, torch.bfloat16, torch.float16, torch.float64):
        ref_agg = None
        for i, u in enumerate(ups):                           # fedbuff.py:94-96,136-157
            ref_agg = torch_cpu.fedbuff_step(ref_agg, {"k": u}, 10, 10 - i)
        w0 = _rand(g, model_dt, 2051, 1.0)
        exp = torch_cpu.fedbuff_scale_add({"k": w0.clone()}, ref_agg, 3)["k"]   # fedbuff.py:122-127
        opt, agg = _drop_in("fedbuff"), None
        for i, u in enumerate(ups):
            c = S.SortedCache()
            c["t"] = S.TR({"k": u.to(DEV)}, 1, 10 - i)
            agg = opt.do(agg, c, total=1, version=10)
        new = opt.scale_add_agg_weights({"k": w0.to(DEV)}, agg, 3)
        S.assert_bitwise(f"{model_dt}+={agg_dt}/3", {"k": new["k"]}, {"k": exp})


def test_slab_holds_kernel_keys_beside_narrow_buffers():
    """A model with a bool mask and a uint8 buffer: DeviceUpdateCache(slab) keeps the
    kernel-dtype keys in the tiled slab (MixedSlotWeights) and the buffers beside them;
    FedAvg and FedBuff (+ scale_add) over those entries == torch CPU's own ops, bitwise."""
    from flame_amd import engine
    from flame_amd.ingest import DeviceUpdateCache
    from flame_amd.slab import MixedSlotWeights
    g = torch.Generator().manual_seed(77)
    T = engine.chunk_elems(0)
    shapes = {"w": ((3 * T + 17,), torch.float32), "mask": ((300,), torch.bool), "bf": ((4099,), torch.bfloat16),
              "u8": ((77,), torch.uint8), "nbt": ((), torch.int64), "m": ((33, 65), torch.float32)}

    def model(scale):
        return {k: (_rand(g, dt, 1, scale).reshape(()) if s == () else _rand(g, dt, int(torch.tensor(s).prod()),
                                                                            scale).reshape(s))
                for k, (s, dt) in shapes.items()}
    base = model(1.0)
    ups = [model(1e-1) for _ in range(6)]
    counts = [3 + 4 * i for i in range(6)]
    total = sum(counts)
    # FedAvg: torch CPU reference vs the drop-in over slab-backed entries
    exp = {k: v.clone() for k, v in base.items()}
    for u, c in zip(ups, counts):
        for k in exp:
            _reference(exp[k], u[k], c / total)
    cache = DeviceUpdateCache(device=DEV, placement="slab", capacity=8)
    for i, (u, c) in enumerate(zip(ups, counts)):
        cache[f"e{i}"] = S.TR({k: v.clone() for k, v in u.items()}, c)
    w0 = cache["e0"].weights
    assert isinstance(w0, MixedSlotWeights) and engine.tiled_stride(w0["w"], shapes["w"][0][0])
    assert cache.slab is not None and cache.slab.keys == ["w", "bf", "nbt", "m"]
    del w0
    out = _drop_in("fedavg").do({k: v.to(DEV) for k, v in base.items()}, cache, total=total)
    S.assert_bitwise("fedavg", {k: out[k] for k in out}, exp)
    # FedBuff one arrival per do(), the aggregate read once at the end, then scale_add
    ref = None
    for i, u in enumerate(ups):
        r = 1 / math.sqrt(1 + 10 - (10 - i % 3))
        tmps = {k: (v * r).to(v.dtype) for k, v in u.items()}
        if ref is None:
            ref = tmps
        else:
            for k in ref:
                ref[k] += tmps[k]
    opt, agg = _drop_in("fedbuff"), None
    for i, u in enumerate(ups):
        c = DeviceUpdateCache(device=DEV, placement="slab", capacity=2) if i == 0 else cache
        c[f"t{i}"] = S.TR({k: v.clone() for k, v in u.items()}, 1, 10 - i % 3)
        agg = opt.do(agg, c, total=1, version=10)
    S.assert_bitwise("fedbuff agg", {k: agg[k] for k in agg}, ref)
    fl = [k for k, (_, dt) in shapes.items() if dt.is_floating_point]
    w = {k: base[k].clone() for k in fl}
    for k in fl:
        w[k] += ref[k] / 6
    new = opt.scale_add_agg_weights({k: base[k].to(DEV) for k in fl}, agg, 6)
    S.assert_bitwise("scale_add", {k: new[k] for k in fl}, w)


def test_sync_hierarchy_with_narrow_buffers_vs_oracle():
    """The synchronous hierarchy over a model with a uint8 buffer and an int16 buffer next
    to f32 / bf16 keys: the fused kernel keys and the composed narrow keys == the oracle's
    op sequence (middle FedAvg, delta new - old, the top's FedAvg of the deltas), bitwise."""
    from flame_amd.optimizer.sync_hierarchy import sync_hierarchy_round
    g = torch.Generator().manual_seed(61)
    shapes = {"w": ((3001,), torch.float32), "bf": ((515,), torch.bfloat16), "u8": ((77,), torch.uint8),
              "i16": ((33,), torch.int16)}

    def model(scale):
        return {k: _rand(g, dt, s[0], scale) for k, (s, dt) in shapes.items()}
    M, C = 5, 3
    mids = [model(1.0) for _ in range(M)]
    ups = [[model(1e-1) for _ in range(C)] for _ in range(M)]
    counts = [[2 + m + 3 * t for t in range(C)] for m in range(M)]
    top = model(1.0)

    def run(dev, fn):
        mw = [{k: v.clone().to(dev) for k, v in w.items()} for w in mids]
        tw = {k: v.clone().to(dev) for k, v in top.items()}
        middles = []
        for m in range(M):
            c = S.SortedCache()
            for t in range(C):
                c[f"t{t}"] = S.TR({k: v.clone().to(dev) for k, v in ups[m][t].items()}, counts[m][t])
            middles.append((mw[m], c, sum(counts[m])))
        tw, deltas = fn(middles, tw, with_delta=True)
        return S.to_cpu(tw), [S.to_cpu(d) for d in deltas], [S.to_cpu(w) for w in mw]
    got = run(DEV, sync_hierarchy_round)
    exp = run("cpu", S.oracle_sync_hierarchy_round)
    S.assert_bitwise("top", got[0], exp[0])
    for m in range(M):
        S.assert_bitwise(f"delta m{m}", got[1][m], exp[1][m])
        S.assert_bitwise(f"mid m{m}", got[2][m], exp[2][m])


@pytest.mark.parametrize("sort", ["fedadam", "fedadagrad"])
def test_fedopt_with_narrow_buffers_vs_oracle(sort):
    """FedOPT over a model with uint8 / int16 buffers next to f32 / bf16 keys, 3 rounds: the
    reduction in the kernels (narrow keys: fp32 tmp + cast, wrapping adds), the adaptive step
    of the narrow keys as the reference's torch op sequence (their d, m, v, current promote
    to fp32) -- against the oracle within the SURVEY §8(c) FedOPT contract."""
    from oracle import oracle as O
    g = torch.Generator().manual_seed(71)
    shapes = {"w": ((2049,), torch.float32), "bf": ((300,), torch.bfloat16), "u8": ((65,), torch.uint8),
              "i16": ((33,), torch.int16)}

    def model(scale):
        return {k: _rand(g, dt, s[0], scale) for k, (s, dt) in shapes.items()}
    hyper = dict(beta_1=0.9, beta_2=0.99, eta=1e-2, tau=1e-3)
    ora = O.OracleFedOPT(sort, **hyper)
    from flame_amd.optimizers import optimizer_provider
    amd = optimizer_provider.get(sort, **hyper)
    w = model(1.0)
    wa, wo = {k: v.to(DEV) for k, v in w.items()}, {k: v.clone() for k, v in w.items()}
    for rnd in range(3):
        ups = [model(1e-1) for _ in range(4)]
        ca, co = S.SortedCache(), S.SortedCache()
        for i, u in enumerate(ups):
            ca[f"e{i}"] = S.TR({k: v.to(DEV) for k, v in u.items()}, 5 + i)
            co[f"e{i}"] = S.TR({k: v.clone() for k, v in u.items()}, 5 + i)
        wa = amd.do({k: v.clone() for k, v in wa.items()}, ca, total=26)
        wo = ora.do({k: v.clone() for k, v in wo.items()}, co, total=26)
        got = S.to_cpu(wa)
        for k in shapes:
            assert got[k].dtype == wo[k].dtype, (rnd, k, got[k].dtype, wo[k].dtype)
            if got[k].is_floating_point():
                # int16's d**2 wraps negative in the reference, so sqrt(v) is NaN there: the
                # NaNs must land where the oracle's do; the rest is checked by the contract
                nan = torch.isnan(wo[k])
                assert torch.equal(torch.isnan(got[k]), nan), (sort, rnd, k)
                got[k] = got[k].masked_fill(nan, 0)
        exp = {k: (v.masked_fill(torch.isnan(v), 0) if v.is_floating_point() else v) for k, v in wo.items()}
        S.assert_close_fedopt(f"{sort} r{rnd}", got, exp, elementwise=(rnd < 2))


def test_narrow_buffers_under_float64_default_dtype():
    """torch.set_default_dtype(torch.float64): the reference's ``(v * rate)`` on a bool / uint8 /
    int8 / int16 buffer is then fp64 (rate unrounded) -- the drop-in's tmp follows the default
    dtype (engine.tmp_of); FedAvg bitwise vs torch CPU, the default restored after."""
    old = torch.get_default_dtype()
    g = torch.Generator().manual_seed(31)
    try:
        torch.set_default_dtype(torch.float64)
        for dt in (torch.bool, torch.uint8, torch.int8, torch.int16):
            acc = _rand(g, dt, 4099, 1.0)
            vs = [_rand(g, dt, 4099, 1e-1) for _ in range(3)]
            counts = [5, 11, 17]
            exp = acc.clone()
            for v, c in zip(vs, counts):
                _reference(exp, v, c / sum(counts))
            cache = S.SortedCache()
            for i, (v, c) in enumerate(zip(vs, counts)):
                cache[f"{i}"] = S.TR({"x": v.to(DEV)}, c)
            got = _drop_in("fedavg").do({"x": acc.to(DEV)}, cache, total=sum(counts))
            assert got["x"].dtype == dt and torch.equal(got["x"].cpu(), exp), dt
    finally:
        torch.set_default_dtype(old)
