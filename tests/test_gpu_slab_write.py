"""Slab inserts through the C ABI (``flame_slab_write`` / ``flame_slab_write_2d``): the role's
``self.cache[end] = tres`` (syncfl/top_aggregator.py:154-156) landing an update in a tiled
UpdateSlab slot.  Every byte of every key must arrive, ragged last tiles and all, from device
sources (contiguous, strided, misaligned views), pinned and pageable host sources; bytes of
other slots and the padding past a key's last element are never touched."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")


def _model(g):
    return {
        "a": torch.randn(3, 1000, generator=g),                          # 3,000 f32: ragged (2 tiles + 952)
        "b": torch.randn(2048, generator=g),                             # exactly 2 f32 tiles
        "c": torch.randn(5, 7, generator=g).to(torch.bfloat16),          # 35 bf16: one partial tile
        "d": torch.randn(4099, generator=g).to(torch.float16),           # f16: 2 tiles + 3
        "e": torch.randint(-2**40, 2**40, (777,), generator=g),          # int64
        "f": torch.tensor(5),                                            # 0-d int64 buffer
        "g": torch.randn(0, generator=g),                                # empty key
        "h": torch.randn(1, generator=g, dtype=torch.float64),           # one f64
        "i": torch.randint(-2**30, 2**30, (1025,), generator=g, dtype=torch.int32),
    }


def _bits(t):
    t = t.reshape(-1)
    return t.view(torch.int16) if t.dtype in (torch.bfloat16, torch.float16) else t


def _check(slab, slot, w):
    for k, v in w.items():
        got = slab.read(slot, k).cpu()
        assert got.dtype == v.dtype and got.shape == v.shape, k
        assert torch.equal(_bits(got), _bits(v.cpu())), k


def test_slab_write_sources_bitwise():
    from flame_amd.slab import UpdateSlab
    g = torch.Generator().manual_seed(5)
    tmpl = _model(g)
    slab = UpdateSlab(tmpl, capacity=6, device=DEV)
    for dt, s in slab.storage.items():      # sentinel: detect writes outside the slot / past numel
        s.view(torch.uint8).fill_(0xA5)
    ups = [_model(g) for _ in range(6)]
    srcs = [
        {k: v.to(DEV) for k, v in ups[0].items()},                                  # device
        {k: v.pin_memory() for k, v in ups[1].items()},                             # pinned host
        {k: v.clone() for k, v in ups[2].items()},                                  # pageable host
        # device, misaligned: every key a view starting one element into a larger buffer
        {k: torch.cat([v.reshape(-1)[:1], v.reshape(-1)]).to(DEV)[1:].view(v.shape) if v.numel() else v.to(DEV)
         for k, v in ups[3].items()},
        # device, non-contiguous (transposed) where the shape allows
        {k: (v.t().contiguous().to(DEV).t() if v.dim() == 2 else v.to(DEV)) for k, v in ups[4].items()},
        # host, misaligned pageable views
        {k: torch.cat([v.reshape(-1)[:1], v.reshape(-1)])[1:].view(v.shape) if v.numel() else v
         for k, v in ups[5].items()},
    ]
    ws = [slab.put(s) for s in srcs]
    torch.cuda.synchronize()
    for w, u in zip(ws, ups):
        _check(slab, w.slot, u)
    # untouched bytes: every slot's padding past numel in its last tile, and no slot beyond 6
    for k in tmpl:
        dt, _, n, tile0, tiles = slab.meta[k]
        T = slab.storage[dt].shape[2]
        if n % T:
            pad = slab.storage[dt][tile0 + tiles - 1, :, n % T:].contiguous().view(torch.uint8)
            assert bool((pad == 0xA5).all()), k


def test_slab_write_reuses_slot_after_release():
    """A slot freed by dropping its weights is rewritten only after the consuming stream passes."""
    from flame_amd.slab import UpdateSlab
    g = torch.Generator().manual_seed(6)
    tmpl = _model(g)
    slab = UpdateSlab(tmpl, capacity=1, device=DEV)
    for r in range(3):
        u = _model(g)
        w = slab.put({k: v.to(DEV) for k, v in u.items()})
        torch.cuda.synchronize()
        _check(slab, w.slot, u)
        del w


def test_slab_write_one_launch_per_update():
    """A device-sourced insert of a 9-key model is one kernel launch (torch's copy_ into the
    strided view used to split it into many)."""
    from flame_amd.slab import UpdateSlab
    from torch.profiler import ProfilerActivity, profile
    g = torch.Generator().manual_seed(7)
    tmpl = _model(g)
    slab = UpdateSlab(tmpl, capacity=4, device=DEV)
    src = {k: v.to(DEV) for k, v in _model(g).items()}
    slab.put(src)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CUDA], acc_events=True) as prof:
        w = slab.put(src)
        torch.cuda.synchronize()
    names = [e.name for e in prof.events() if e.device_type.name == "CUDA"]
    launches = [n for n in names if "slab_write_kernel" in n]
    assert len(launches) == 1, names
    assert not [n for n in names if "copy" in n.lower()], names
    _check(slab, w.slot, {k: v.cpu() for k, v in src.items()})


def test_slab_write_entry_points_direct():
    """The C entry points on a raw table: >89 entries split over launches, device sources at every
    16-byte misalignment, 2D copies from host."""
    from flame_amd import _native as N
    L = N.lib()
    n_ent, stride = 200, 3 * N.FLAME_TILE_BYTES
    g = torch.Generator().manual_seed(8)
    sizes = [int(x) for x in torch.randint(0, 3 * N.FLAME_TILE_BYTES, (n_ent,), generator=g)]
    dst = torch.zeros(n_ent, 3, 3, N.FLAME_TILE_BYTES, dtype=torch.uint8, device=DEV)   # [entry][tile][slot][bytes]
    srcs = [torch.randint(0, 256, (s,), generator=g, dtype=torch.uint8) for s in sizes]
    # device sources at every misalignment 0..15 (the kernel's funnel-shift path)
    dsrc = []
    for i, s in enumerate(srcs):
        o = i % 16
        buf = torch.zeros(s.numel() + 16, dtype=torch.uint8, device=DEV)
        buf[o:o + s.numel()] = s.to(DEV)
        dsrc.append(buf[o:o + s.numel()])
    tab = np.zeros((n_ent, 4), dtype=np.int64)
    for i, s in enumerate(dsrc):
        tab[i] = (s.data_ptr(), dst[i, 0, 1].data_ptr(), sizes[i], stride)
    N.check(L.flame_slab_write(tab.ctypes.data, n_ent, torch.cuda.current_stream().cuda_stream))
    host = [s.pin_memory() for s in srcs]
    for i, s in enumerate(host):
        tab[i] = (s.data_ptr(), dst[i, 0, 2].data_ptr(), sizes[i], stride)
    N.check(L.flame_slab_write_2d(tab.ctypes.data, n_ent, torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    out = dst.cpu()
    for i, s in enumerate(srcs):
        for slot in (1, 2):
            got = out[i, :, slot, :].reshape(-1)
            assert torch.equal(got[:sizes[i]], s), (i, slot)
            assert int(got[sizes[i]:].sum()) == 0, (i, slot)
        assert int(out[i, :, 0, :].sum()) == 0
    # argument checks
    bad = np.array([[dsrc[0].data_ptr(), dst.data_ptr() + 1, 100, stride]], dtype=np.int64)
    assert L.flame_slab_write(bad.ctypes.data, 1, None) == N.FLAME_EINVAL
    bad[0, 1], bad[0, 2], bad[0, 3] = dst.data_ptr(), 2 * N.FLAME_TILE_BYTES, 100
    assert L.flame_slab_write(bad.ctypes.data, 1, None) == N.FLAME_EINVAL
    assert b"dst_tile_stride" in L.flame_last_error()


@pytest.mark.oracle
def test_decoded_payloads_one_transfer_each_and_pinned_ring():
    """Channel payloads decoded zero-copy (ingest.decode) into a slab-placed DeviceUpdateCache:
    each update's tensors -- views into one pageable payload -- cross PCIe as ONE span, staged
    through the slab's pinned ring (more payloads than ring slots); the payload buffers are
    overwritten right after each insert (the receiver reuses them), and the FedAvg over the
    cache still equals the oracle on the original bytes, bitwise."""
    import cloudpickle
    import scenarios as S
    from flame_amd import ingest
    from flame_amd.optimizers import optimizer_provider
    from flame_amd.slab import PINNED_RING, PINNED_STAGE_MIN
    from oracle import oracle as O
    g = torch.Generator().manual_seed(12)
    shapes = {"conv.w": (32, 1, 3, 3), "conv.b": (32,), "fc.w": (128, 2304), "fc.b": (128,), "out.w": (10, 128),
              "bn": (64,)}
    n = PINNED_RING + 3
    ups = [{k: torch.randn(s, generator=g) * 1e-2 for k, s in shapes.items()} for _ in range(n)]
    base = {k: torch.randn(s, generator=g) for k, s in shapes.items()}
    counts = [100 + 7 * i for i in range(n)]
    cache = ingest.DeviceUpdateCache(device=DEV, placement="slab", capacity=n)
    for i, u in enumerate(ups):
        buf = bytearray(cloudpickle.dumps({"weights": u, "dataset_size": counts[i]}))
        assert len(buf) > PINNED_STAGE_MIN
        msg = ingest.decode(buf)
        assert all(getattr(v, "_flame_payload", None) is buf for v in msg["weights"].values())
        cache[f"t{i}"] = S.TR(msg["weights"], counts[i])
        assert getattr(cache[f"t{i}"].weights, "slab", None) is not None
        buf[:] = b"\xff" * len(buf)            # the receive buffer is reused for the next message
    got = optimizer_provider.get("fedavg").do({k: v.to(DEV) for k, v in base.items()}, cache, total=sum(counts))
    exp = {k: v.clone() for k, v in base.items()}
    co = S.SortedCache()
    for i, u in enumerate(ups):
        co[f"t{i}"] = S.TR({k: v.clone() for k, v in u.items()}, counts[i])
    O.OracleFedAvg().do(exp, co, total=sum(counts))
    S.assert_bitwise("payload-staged fedavg", S.to_cpu(got), exp)


@pytest.mark.parametrize("offset", [1, 3, 4, 8])
def test_misaligned_pinned_host_source(monkeypatch, offset):
    """A pinned host source that is not 4-byte aligned (a storage inside a pickled payload in a
    LIFL shm segment, or a rank's slice of one) goes through the tile-copy kernel over its
    device-mapped address, not hipMemcpy2DAsync (~5 GB/s there, profiles/r06e2_h2d_paths.log);
    aligned ones keep the pitched DMA.  Bitwise either way, ragged tail included."""
    from flame_amd import _native as N
    from flame_amd.slab import UpdateSlab
    real = N.lib()
    calls = []

    class Spy:
        def __getattr__(self, name):
            fn = getattr(real, name)
            if name in ("flame_slab_write", "flame_slab_write_2d"):
                def wrapped(*a):
                    calls.append(name)
                    return fn(*a)
                return wrapped
            return fn
    monkeypatch.setattr(N, "lib", lambda: Spy())
    n = 3 * 1024 + 17
    buf = torch.empty(4 * n + 64, dtype=torch.uint8, pin_memory=True)
    src = torch.frombuffer(buf.numpy(), dtype=torch.float32, offset=offset, count=n)
    src.copy_(torch.randn(n, generator=torch.Generator().manual_seed(offset)))
    assert src.is_pinned() and src.data_ptr() % 4 == offset % 4
    slab = UpdateSlab({"w": torch.empty(n)}, capacity=3, device=DEV)
    slab.put({"w": torch.zeros(n, device=DEV)})
    sw = slab.put({"w": src})
    torch.cuda.synchronize()
    assert torch.equal(slab.read(sw.slot, "w").cpu(), src)
    assert calls[-1] == ("flame_slab_write" if offset % 4 else "flame_slab_write_2d"), calls
