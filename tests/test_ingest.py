"""Zero-copy restricted decoding of flame channel payloads (flame_amd.ingest)."""
import enum
import os
import pickle
import time

import cloudpickle
import numpy as np
import pytest
import torch

from flame_amd import ingest


class MsgType(enum.Enum):  # stand-in for flame.common.constants.MessageType
    WEIGHTS = 1
    DATASET_SIZE = 3
    MODEL_VERSION = 5


def _msg():
    g = torch.Generator().manual_seed(0)
    big = torch.randn(64, 33, generator=g)
    return {
        MsgType.WEIGHTS: {
            "conv.weight": torch.randn(16, 3, 3, 3, generator=g),
            "bias": torch.randn(16, generator=g).to(torch.bfloat16),
            "half": torch.randn(7, generator=g).half(),
            "dbl": torch.randn(5, generator=g).double(),
            "nbt": torch.tensor(12345678901, dtype=torch.int64),
            "i32": torch.arange(10, dtype=torch.int32),
            "mask": torch.tensor([True, False, True]),
            "empty": torch.empty(0, 4),
            "slice": big[5:9],            # storage offset != 0
            "transposed": big.t(),         # non-contiguous strides
        },
        MsgType.DATASET_SIZE: 2000,
        MsgType.MODEL_VERSION: 7,
        "meta": {"ratio": 0.5, "name": "trainer-1", "tags": ["a", "b"], "none": None, "pair": (1, 2.5)},
    }


def _same(a, b):
    assert a.dtype == b.dtype and a.shape == b.shape and a.stride() == b.stride() or a.numel() == 0
    if a.dtype == torch.bfloat16:
        a, b = a.view(torch.int16), b.view(torch.int16)
    assert torch.equal(a, b)


def test_decode_matches_cloudpickle_and_is_zero_copy():
    msg = _msg()
    payload = cloudpickle.dumps(msg)
    out = ingest.decode(payload, extra_globals=ingest.allow_enum(MsgType))
    ref = cloudpickle.loads(payload)
    assert out[MsgType.DATASET_SIZE] == 2000 and out[MsgType.MODEL_VERSION] == 7
    assert out["meta"] == ref["meta"]
    base = np.frombuffer(payload, dtype=np.uint8).ctypes.data
    for k, v in ref[MsgType.WEIGHTS].items():
        got = out[MsgType.WEIGHTS][k]
        _same(got, v)
        if got.numel():
            assert base <= got.data_ptr() < base + len(payload), f"{k} was copied"


def test_decode_refuses_arbitrary_globals():
    class Evil:
        def __reduce__(self):
            return (os.system, ("true",))
    with pytest.raises(pickle.UnpicklingError):
        ingest.decode(pickle.dumps({"x": Evil()}, protocol=5))
    with pytest.raises(pickle.UnpicklingError):
        ingest.decode(cloudpickle.dumps({"f": lambda x: x}))
    # the channel-level loads() falls back to the reference decoder for non-update messages
    assert ingest.loads(cloudpickle.dumps({"f": 1.5}))["f"] == 1.5


def test_decode_protocols_and_large_update_speed():
    w = {"fc.weight": torch.randn(1 << 22)}    # 16 MB
    for proto in (2, 4, 5):
        payload = pickle.dumps({"w": w, "n": 3}, protocol=proto)
        out = ingest.decode(payload)
        assert torch.equal(out["w"]["fc.weight"], w["fc.weight"]) and out["n"] == 3
    payload = cloudpickle.dumps({"w": w})
    t0 = time.perf_counter()
    for _ in range(5):
        ingest.decode(payload)
    t_dec = (time.perf_counter() - t0) / 5
    t0 = time.perf_counter()
    for _ in range(5):
        cloudpickle.loads(payload)
    t_ref = (time.perf_counter() - t0) / 5
    assert t_dec < t_ref, (t_dec, t_ref)


def test_device_update_cache_host_placement_orders_and_pops():
    from scenarios import TR
    c = ingest.DeviceUpdateCache(placement="host")  # host placement needs no GPU
    for k in ["b", "a", "c"]:
        c[k] = TR({"w": torch.ones(3)}, 1)
    assert len(c) == 3 and list(c.iterkeys()) == ["a", "b", "c"] and "a" in c
    t = c.pop("a")
    assert t.count == 1 and len(c) == 2 and c.pop("zz") is None


def test_decode_malformed_payloads_raise_unpickling_error():
    payload = cloudpickle.dumps({"w": torch.randn(100)})
    for bad in (payload[:len(payload) // 2], payload[:10], b"\x80\x05\xff", b""):
        with pytest.raises(pickle.UnpicklingError):
            ingest.decode(bad)


def test_decode_property_random_messages():
    """Property: for random update-like messages, decode == cloudpickle.loads (values, dtypes,
    shapes, strides) -- hypothesis-generated dtypes, shapes, views and metadata."""
    from hypothesis import given, settings, strategies as st

    dts = st.sampled_from([torch.float32, torch.bfloat16, torch.float16, torch.float64, torch.int64,
                           torch.int32, torch.uint8, torch.bool])
    shapes = st.lists(st.integers(0, 7), min_size=0, max_size=3)

    @settings(max_examples=60, deadline=None)
    @given(dts, shapes, st.integers(0, 3), st.dictionaries(st.text(max_size=5), st.integers() | st.floats(
        allow_nan=False) | st.text(max_size=8) | st.none(), max_size=4), st.booleans())
    def check(dt, shape, off, meta, transpose):
        base = (torch.arange(int(np.prod(shape or [1])) + off) % 5).to(dt)
        t = base[off:].reshape(shape) if shape else base[off:off + 1].reshape(())
        if transpose and t.dim() >= 2:
            t = t.transpose(0, 1)
        payload = cloudpickle.dumps({"weights": {"t": t}, "meta": meta})
        got = ingest.decode(payload)
        ref = cloudpickle.loads(payload)
        assert got["meta"] == ref["meta"]
        g, r = got["weights"]["t"], ref["weights"]["t"]
        assert g.dtype == r.dtype and g.shape == r.shape and g.stride() == r.stride()
        if dt == torch.bfloat16:
            g, r = g.view(torch.int16), r.view(torch.int16)
        assert torch.equal(g, r)
    check()


def test_shm_receiver_decodes_in_place():
    """ShmReceiver (backend/shm.py:386-391 stand-in) decodes a message in the sender's
    segment without copying: the tensors alias the shared memory."""
    import numpy as np
    from multiprocessing import shared_memory
    w = {"w": torch.arange(1000, dtype=torch.float32), "b": torch.ones(3, dtype=torch.bfloat16)}
    blob = cloudpickle.dumps({"weights": w, "dataset_size": 77})
    seg = shared_memory.SharedMemory(name="flametest_a-agg", create=True, size=len(blob) + 64)
    try:
        seg.buf[:len(blob)] = blob
        rx = ingest.ShmReceiver("agg", register=False, untrack=False)   # same process as the writer
        msg = rx.loads("flametest_a", len(blob))
        assert msg["dataset_size"] == 77
        assert torch.equal(msg["weights"]["w"], w["w"]) and torch.equal(msg["weights"]["b"], w["b"])
        mapping = rx._segs["flametest_a-agg"][0].buf
        base = np.frombuffer(mapping, dtype=np.uint8).ctypes.data
        assert base <= msg["weights"]["w"].data_ptr() < base + len(mapping)   # a view, not a copy
        del mapping
        del msg
        rx.close()
    finally:
        seg.close()
        seg.unlink()


def test_shm_lease_registry_and_generations():
    """flame_amd.shm_lease: address ranges of open segments, message generations, and the
    stale-view check the consumers apply (no GPU: an unregistered receiver)."""
    import cloudpickle
    from multiprocessing import shared_memory
    from flame_amd import ingest, shm_lease
    w = {"w": torch.arange(1000, dtype=torch.float32)}
    blob = cloudpickle.dumps({"weights": w, "dataset_size": 3})
    seg = shared_memory.SharedMemory(name="flamelease_cpu-agg", create=True, size=len(blob) + 64)
    try:
        seg.buf[:len(blob)] = blob
        rx = ingest.ShmReceiver("agg", register=False, untrack=False)
        m1 = rx.loads("flamelease_cpu", len(blob))
        t = m1["weights"]["w"]
        assert shm_lease.aliases(t) and shm_lease.segment_of(t.data_ptr()) == "flamelease_cpu-agg"
        assert not shm_lease.aliases(torch.zeros(4))
        shm_lease.check_live(t)                       # current message: fine
        shm_lease.check_live(t.reshape(-1)[:10])      # untagged derived view: not checked
        m2 = rx.loads("flamelease_cpu", len(blob))    # the sender's next message
        shm_lease.check_live(m2["weights"]["w"])
        with pytest.raises(RuntimeError, match="stale"):
            shm_lease.check_live(t)
        del m1, m2, t
        rx.close()
        assert shm_lease.segment_of(np.frombuffer(seg.buf, dtype=np.uint8).ctypes.data) is None
    finally:
        seg.close()
        seg.unlink()


def test_storage_records_parsed_without_the_vm(monkeypatch):
    """Every storage record torch's legacy save writes -- its key is the trainer's storage
    ADDRESS, new in every message -- is parsed by the strict field-by-field parser
    (ingest._parse_storage_record), for every dtype and numel encoding (BININT1 / BININT2 /
    BININT / LONG1); a record that departs from the layout in any byte goes to the restricted
    VM, which still refuses what it does not allow."""
    import pickle
    import cloudpickle
    from flame_amd import ingest

    def no_slow(mv, q):
        raise AssertionError("the one-match record parser should have taken this record")
    monkeypatch.setattr(ingest, "_parse_storage_record_slow", no_slow)
    g = torch.Generator().manual_seed(4)
    for dt in (torch.float32, torch.bfloat16, torch.float16, torch.float64, torch.int64, torch.int32, torch.int16,
               torch.int8, torch.uint8, torch.bool):
        for n in (1, 200, 300, 70_000, 3_000_001):
            t = (torch.randn(n, generator=g) * 50).to(dt)
            payload = cloudpickle.dumps({"weights": {"w": t, "v": t[1:]}, "dataset_size": 7})
            ingest._STORAGE_RECORDS.clear()
            got = ingest.decode(payload)["weights"]
            assert torch.equal(got["w"], t) and torch.equal(got["v"], t[1:]), (dt, n)
            assert not ingest._STORAGE_RECORDS, (dt, n)        # the fast parser took every record
    monkeypatch.undo()
    # the field-by-field parser agrees with the one-match parser on every record above
    for dt in (torch.float32, torch.bfloat16, torch.int64, torch.bool):
        t = torch.ones(300_001, dtype=dt)
        payload = cloudpickle.dumps({"w": t})
        mv = memoryview(payload)
        q = payload.find(b"\x80\x02(X\x07\x00\x00\x00storage")
        assert ingest._parse_storage_record(mv, q) == ingest._parse_storage_record_slow(mv, q) != None
    # a record naming a storage type outside the allowlist: fast parser declines, the VM refuses
    t = torch.ones(4)
    payload = bytearray(cloudpickle.dumps({"w": t}))
    i = payload.find(b"torch\nFloatStorage\n")
    payload[i:i + len(b"torch\nFloatStorage\n")] = b"torch\nFloatXtorage\n"
    with pytest.raises(pickle.UnpicklingError):
        ingest.decode(bytes(payload))


def test_storage_record_cache_is_bounded():
    """The VM's record cache is keyed by sender-controlled bytes: long records are never kept,
    and neither the number of distinct lengths nor the entry count can grow past the caps."""
    from flame_amd import ingest
    saved = {k: dict(v) for k, v in ingest._STORAGE_RECORDS.items()}
    ingest._STORAGE_RECORDS.clear()
    try:
        ingest._remember_record(b"x" * (ingest.RECORD_CACHE_MAX_BYTES + 1), (None, 0, 0))
        assert not ingest._STORAGE_RECORDS
        for n in range(1, 3 * ingest.RECORD_CACHE_MAX_LENGTHS):
            ingest._remember_record(b"y" * n, (None, 0, 0))
        assert len(ingest._STORAGE_RECORDS) == ingest.RECORD_CACHE_MAX_LENGTHS
        for i in range(2 * ingest.RECORD_CACHE_MAX_ENTRIES):
            ingest._remember_record(i.to_bytes(4, "little"), (None, 0, 0))
        assert sum(len(v) for v in ingest._STORAGE_RECORDS.values()) == ingest.RECORD_CACHE_MAX_ENTRIES
    finally:
        ingest._STORAGE_RECORDS.clear()
        ingest._STORAGE_RECORDS.update(saved)


def test_decode_does_not_silence_warnings_process_wide():
    """Importing / using the decoder leaves the process's warning filters alone."""
    import warnings
    from flame_amd import ingest  # noqa: F401
    assert not any(f[1] is not None and "not writable" in f[1].pattern for f in warnings.filters
                   if f[1] is not None)
