"""The oracle's per-arrival add against torch CPU itself -- the reference's arithmetic
(fedavg.py:93-104: ``tmp = v * rate; tmp = tmp.to(v.dtype); agg[k] += tmp``) -- for every
pair of (aggregate dtype, update dtype) a state_dict can carry, bitwise, errors included.
No GPU: this pins the restatement the GPU tests compare against."""
import pytest
import torch

from oracle import consult
from oracle import oracle as O

DTYPES = [torch.float32, torch.bfloat16, torch.float16, torch.float64, torch.int64, torch.int32,
          torch.int16, torch.int8, torch.uint8, torch.bool]


def _rand(g, dt, n, scale):
    if dt == torch.bool:
        return torch.rand(n, generator=g) < 0.4
    if dt.is_floating_point:
        return (torch.randn(n, generator=g, dtype=torch.float64) * scale).to(dt)
    hi = {torch.uint8: 200, torch.int8: 100, torch.int16: 30000}.get(dt, 1 << 30)
    lo = 0 if dt == torch.uint8 else -hi
    return torch.randint(lo, hi, (n,), generator=g, dtype=torch.int64).to(dt)


def _reference(acc, v, rate):
    """The reference's add (fedavg.py:93-104) in torch CPU ops: a checker (consult.py)."""
    consult.note()
    tmp = v * rate
    tmp = tmp.to(dtype=v.dtype) if tmp.dtype != v.dtype else tmp
    acc += tmp


@pytest.mark.parametrize("acc_dt", DTYPES, ids=[str(d)[6:] for d in DTYPES])
def test_oracle_add_matches_torch_every_dtype_pair(acc_dt):
    g = torch.Generator().manual_seed(hash(str(acc_dt)) % 1000)
    for v_dt in DTYPES:
        for rate in (0.3712, 1.0, 1 / 3):
            acc = _rand(g, acc_dt, 1031, 1.0)
            v = _rand(g, v_dt, 1031, 1e-1)
            exp, got = acc.clone(), acc.clone()
            try:
                _reference(exp, v, rate)
                err = None
            except RuntimeError as e:
                err = e
            if err is not None:
                with pytest.raises(RuntimeError):
                    O.reduce_tensor(got, [v], [rate])
                continue
            O.reduce_tensor(got, [v], [rate])
            assert torch.equal(got.view(torch.uint8), exp.view(torch.uint8)), (acc_dt, v_dt, rate)


@pytest.mark.parametrize("agg_dt", [torch.float32, torch.bfloat16, torch.float16, torch.float64, torch.int64,
                                    torch.uint8])
def test_oracle_fedbuff_scale_add_every_model_dtype(agg_dt):
    """The oracle FedBuff (None start, staleness rates) + scale_add into a model of every
    float dtype, against torch CPU's own ops (fedbuff.py:96,122-157)."""
    import math
    import scenarios as S
    g = torch.Generator().manual_seed(40)
    ups = [_rand(g, agg_dt, 2051, 1e-1) for _ in range(3)]
    for model_dt in (torch.float32, torch.bfloat16, torch.float16, torch.float64):
        ref = None
        for i, u in enumerate(ups):
            tmp = u * (1 / math.sqrt(1 + 10 - (10 - i)))
            tmp = tmp.to(u.dtype) if tmp.dtype != u.dtype else tmp
            if ref is None:
                ref = tmp
            else:
                ref += tmp
        w0 = _rand(g, model_dt, 2051, 1.0)
        exp = w0.clone()
        exp += ref / 3
        opt, agg = O.OracleFedBuff(), None
        for i, u in enumerate(ups):
            c = S.SortedCache()
            c["t"] = S.TR({"k": u}, 1, 10 - i)
            agg = opt.do(agg, c, total=1, version=10)
        new = opt.scale_add_agg_weights({"k": w0.clone()}, agg, 3)
        assert torch.equal(new["k"].view(torch.uint8), exp.view(torch.uint8)), (agg_dt, model_dt)
