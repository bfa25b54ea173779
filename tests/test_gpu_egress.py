"""GPU: the egress encoder over a device-resident aggregated model -- each tensor's bytes go by
ONE D2H copy straight into the pinned payload, and the trainer's ``cloudpickle.loads``
(channel.py:321-325) returns the model bitwise (flame_amd/egress.py)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
cloudpickle = pytest.importorskip("cloudpickle")

DEV = torch.device("cuda:0")


def test_device_model_encodes_by_direct_d2h():
    from flame_amd import egress, ingest
    g = torch.Generator().manual_seed(9)
    model = {"conv1.weight": torch.randn(32, 1, 3, 3, generator=g), "conv1.bias": torch.randn(32, generator=g),
             "fc1.weight": torch.randn(128, 9216, generator=g), "emb": torch.randn(1000, 64, generator=g).bfloat16(),
             "h": torch.randn(4099, generator=g).half(), "nbt": torch.tensor(11), "mask": torch.rand(9, generator=g) > .5}
    dev = {k: v.to(DEV) for k, v in model.items()}
    enc = egress.MessageEncoder(ring=2)
    for r in range(3):       # the ring's buffers are pinned and reused round after round
        for v in dev.values():
            if v.is_floating_point():
                v.add_(1.0)
        for v in model.values():
            if v.is_floating_point():
                v.add_(1.0)
        pl = enc.encode({"weights": dev, "round": r})
        back = cloudpickle.loads(bytes(pl))
        assert back["round"] == r
        for k, v in model.items():
            got = back["weights"][k]
            assert got.dtype == v.dtype and got.shape == v.shape and torch.equal(got, v), (r, k)
        dec = ingest.decode(pl)
        for k, v in model.items():
            assert torch.equal(dec["weights"][k], v), (r, k)
    assert all(b is None or b.is_pinned() for b in enc._bufs)
