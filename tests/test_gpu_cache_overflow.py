"""GPU: a DeviceUpdateCache whose slab is full keeps the overflowing updates as one HBM
tensor per key; a round then mixes tiled slab slots and plain tensors.  FedAvg, FedAdam and
FedBuff (+ scale_add) over such rounds == the same drop-ins over plain device tensors,
bitwise, round after round (slots recycled between rounds)."""
import pytest
import torch

import scenarios as S

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _native_loaded():
    from flame_amd import _native
    _native.lib()
    assert torch.cuda.is_available()


def _get(sort, **kw):
    from flame_amd.optimizers import optimizer_provider
    return optimizer_provider.get(sort, **kw)


def _model(g):
    from flame_amd import engine
    T = engine.chunk_elems(0)
    return {"w": torch.randn(2 * T + 5, generator=g), "bf": torch.randn(4099, generator=g).bfloat16(),
            "m": torch.randn(33, 65, generator=g), "nbt": torch.tensor(4, dtype=torch.int64)}


def _up(g, tmpl, i):
    return {k: (torch.randn(v.shape, generator=g) * 1e-2).to(v.dtype) if v.is_floating_point()
            else torch.tensor(i, dtype=v.dtype) for k, v in tmpl.items()}


@pytest.mark.parametrize("sort", ["fedavg", "fedadam"])
def test_sync_round_with_slab_overflow(sort):
    from flame_amd.ingest import DeviceUpdateCache
    g = torch.Generator().manual_seed(91)
    tmpl = _model(g)
    kw = dict(beta_1=0.9, beta_2=0.99, eta=1e-2, tau=1e-3) if sort == "fedadam" else {}
    a, b = _get(sort, **kw), _get(sort, **kw)
    cache = DeviceUpdateCache(device=DEV, placement="slab", capacity=4)
    wa = {k: v.to(DEV) for k, v in tmpl.items()}
    wb = {k: v.to(DEV) for k, v in tmpl.items()}
    for rnd in range(3):
        n = 9
        ups = [_up(g, tmpl, 10 * rnd + i) for i in range(n)]
        counts = [4 + 3 * i for i in range(n)]
        cb = S.SortedCache()
        for i in range(n):
            cache[f"e{i}"] = S.TR({k: v.clone() for k, v in ups[i].items()}, counts[i])
            cb[f"e{i}"] = S.TR({k: v.to(DEV) for k, v in ups[i].items()}, counts[i])
        kinds = {type(cache[f"e{i}"].weights).__name__ for i in range(n)}
        assert kinds == {"SlotWeights", "dict"}, kinds            # slab slots and overflow tensors
        ra = a.do({k: v.clone() for k, v in wa.items()}, cache, total=sum(counts))
        rb = b.do({k: v.clone() for k, v in wb.items()}, cb, total=sum(counts))
        S.assert_bitwise(f"{sort} r{rnd}", S.to_cpu(ra), S.to_cpu(rb))
        wa, wb = ra, rb


def test_fedbuff_with_slab_overflow():
    from flame_amd.ingest import DeviceUpdateCache
    g = torch.Generator().manual_seed(92)
    tmpl = {k: v for k, v in _model(g).items() if v.is_floating_point()}
    a, b = _get("fedbuff"), _get("fedbuff")
    cache = DeviceUpdateCache(device=DEV, placement="slab", capacity=3)
    held = []
    aa = ab = None
    for i in range(8):
        u = _up(g, tmpl, i)
        cache[f"t{i}"] = S.TR({k: v.clone() for k, v in u.items()}, 1, 20 - i % 4)
        held.append(cache[f"t{i}"])               # queued arrivals keep their slots: later ones overflow
        cb = S.SortedCache()
        cb[f"t{i}"] = S.TR({k: v.to(DEV) for k, v in u.items()}, 1, 20 - i % 4)
        one = S.SortedCache()
        one[f"t{i}"] = cache.pop(f"t{i}")
        aa = a.do(aa, one, total=1, version=20)
        ab = b.do(ab, cb, total=1, version=20)
    wa = {k: (torch.randn(v.shape, generator=g)).to(v.dtype).to(DEV) for k, v in tmpl.items()}
    wb = {k: v.clone() for k, v in wa.items()}
    a.scale_add_agg_weights(wa, aa, 8)
    b.scale_add_agg_weights(wb, ab, 8)
    S.assert_bitwise("fedbuff agg", S.to_cpu(aa), S.to_cpu(ab))
    S.assert_bitwise("fedbuff scale_add", S.to_cpu(wa), S.to_cpu(wb))
