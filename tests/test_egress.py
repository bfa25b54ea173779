"""The egress encoder (flame_amd/egress.py): the aggregated model as the payload flame's channel
sends back to every trainer (syncfl/top_aggregator.py:184-215 -> channel.py:203-218).

Pinned to the reference's own formats: ``cloudpickle.loads`` (what the trainer's channel runs,
channel.py:321-325) returns an equal message, the restricted decoder too, and every storage
stream header is byte-for-byte what torch's legacy save writes for the same storage."""
import enum
import io
import warnings

import numpy as np
import pytest
import torch

cloudpickle = pytest.importorskip("cloudpickle")


class Kind(enum.Enum):
    WEIGHTS = 0
    ROUND = 1


def _model(g):
    return {
        "conv.w": torch.randn(32, 1, 3, 3, generator=g),
        "conv.b": torch.randn(32, generator=g).bfloat16(),
        "fc.w": torch.randn(10, 300, generator=g).half(),
        "bn.n": torch.tensor(7),
        "mask": torch.rand(17, generator=g) > 0.3,
        "empty": torch.randn(0, generator=g),
        "t": torch.randn(12, 9, generator=g).t(),                 # non-contiguous
        "view": torch.randn(1000, generator=g).double()[5:300:7],  # a strided view of a bigger storage
        "i32": torch.randint(-9, 9, (33,), generator=g, dtype=torch.int32),
        "u8": torch.randint(0, 255, (5, 5), generator=g, dtype=torch.uint8),
    }


def _eq(a, b):
    return a.dtype == b.dtype and a.shape == b.shape and torch.equal(a, b)


def test_encode_roundtrips_through_cloudpickle_and_the_decoder():
    from flame_amd import egress, ingest
    g = torch.Generator().manual_seed(1)
    w = _model(g)
    msg = {Kind.WEIGHTS: w, Kind.ROUND: 12, "meta": {"sizes": [3, 4], "x": (1.5, None, "s")}, "alias": w["conv.w"]}
    enc = egress.MessageEncoder(ring=2, pin=False)
    pl = enc.encode(msg)
    back = cloudpickle.loads(bytes(pl))
    assert back[Kind.ROUND] == 12 and back["meta"] == msg["meta"]
    assert back["alias"] is back[Kind.WEIGHTS]["conv.w"]            # a shared tensor stays shared
    for k, v in w.items():
        assert _eq(back[Kind.WEIGHTS][k], v), k
    raw = bytes(pl)
    dec = ingest.decode(raw, extra_globals=ingest.allow_enum(Kind))
    origin = torch.frombuffer(raw, dtype=torch.uint8).data_ptr()
    for k, v in w.items():
        got = dec[Kind.WEIGHTS][k]
        assert _eq(got, v), k
        if v.numel():
            assert (got.data_ptr() - origin) % 64 == 0, k            # raw bytes 64-byte aligned in the payload
    # a second encode on the ring leaves the first payload intact (ring of 2)
    pl2 = enc.encode({"w": torch.zeros(3)})
    assert _eq(cloudpickle.loads(bytes(pl))[Kind.WEIGHTS]["fc.w"], w["fc.w"])
    assert _eq(cloudpickle.loads(bytes(pl2))["w"], torch.zeros(3))


def test_storage_stream_head_is_torchs_own_bytes():
    """For the canonical encodings the head equals what torch's legacy save of that storage
    writes, byte for byte (key = torch's own key for it)."""
    from flame_amd import egress
    g = torch.Generator().manual_seed(2)
    for dt in (torch.float32, torch.bfloat16, torch.float16, torch.float64, torch.int64, torch.int32, torch.int16,
               torch.int8, torch.uint8, torch.bool):
        for n in (1, 255, 256, 65535, 65536, 3_000_001):
            t = (torch.randn(n, generator=g) * 9).to(dt)
            bio = io.BytesIO()
            with warnings.catch_warnings():
                warnings.simplefilter("ignore")
                st = t.storage()
                torch.save(st, bio, _use_new_zipfile_serialization=False)
                key = str(st._untyped_storage._cdata)
            s = bio.getvalue()
            head = egress.storage_stream_head(dt, n, key)
            assert s[:len(head)] == head, (dt, n)
            assert len(s) == len(head) + n * t.element_size(), (dt, n)


def test_encode_refuses_non_weights():
    from flame_amd import egress
    with pytest.raises(TypeError):
        egress.MessageEncoder(pin=False).encode({"w": torch.ones(3, requires_grad=True)})
    with pytest.raises(TypeError):
        egress.MessageEncoder(pin=False).encode({"w": torch.ones(3, dtype=torch.complex64)})


def test_dumps_matches_cloudpickle_semantics_property():
    """Random nested messages: cloudpickle.loads(egress.dumps(m)) == cloudpickle.loads(cloudpickle.dumps(m))."""
    from flame_amd import egress
    rng = np.random.default_rng(3)
    dts = [torch.float32, torch.bfloat16, torch.float16, torch.int64, torch.bool]
    for trial in range(25):
        w = {}
        for k in range(int(rng.integers(1, 6))):
            shape = tuple(int(x) for x in rng.integers(0, 5, size=int(rng.integers(0, 4))))
            dt = dts[int(rng.integers(len(dts)))]
            t = torch.from_numpy(rng.standard_normal(shape).astype(np.float32)).to(dt) if shape else \
                torch.tensor(float(rng.standard_normal())).to(dt)
            w[f"k{k}"] = t
        msg = {"weights": w, "n": int(rng.integers(0, 1 << 40)), "tag": [trial, "x"]}
        a = cloudpickle.loads(egress.dumps(msg))
        b = cloudpickle.loads(cloudpickle.dumps(msg))
        assert a["n"] == b["n"] and a["tag"] == b["tag"]
        for k in w:
            assert _eq(a["weights"][k], b["weights"][k]), (trial, k)
