"""Lifetime of zero-copy views into LIFL shared-memory segments (flame_amd.shm_lease).

The sender rewrites its segment for its next message (backend/shm.py:393-403) at a
time the receiver does not learn; the reference copies every message out on arrival
(:386-391).  Every consumer of ShmReceiver's in-place views must therefore be done
with the segment when its call returns.  Each test rewrites the segment with the
sender's next message right after the consuming call and checks the aggregate is the
oracle's on the FIRST message.
"""
import os

import cloudpickle
import pytest
import torch

import scenarios as S

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
P = 8_000_003          # 32 MB per update: a PCIe read long enough to race a rewrite


@pytest.fixture(scope="module", autouse=True)
def _native_loaded():
    from flame_amd import _native
    _native.lib()
    torch.empty(1, device=DEV)


class _Sender:
    """One trainer's segment ``<tag>-agg``: ``send`` rewrites it in place, as the backend does."""

    def __init__(self, tag, nbytes):
        from multiprocessing import shared_memory
        self.tag = tag
        self.seg = shared_memory.SharedMemory(name=f"{tag}-agg", create=True, size=nbytes)

    def send(self, msg):
        blob = cloudpickle.dumps(msg)
        self.seg.buf[:len(blob)] = blob
        return len(blob)

    def close(self):
        self.seg.close()
        self.seg.unlink()


def _msgs(seed, n=2):
    g = torch.Generator().manual_seed(seed)
    return [{"weights": {"w": torch.randn(P, generator=g) * 1e-2, "b": torch.randn(37, generator=g)},
             "dataset_size": 10 + i} for i in range(n)]


def _run(consume):
    from flame_amd import ingest
    m1, m2 = _msgs(71)
    tag = f"flamelease{os.getpid()}"
    snd = _Sender(tag, len(cloudpickle.dumps(m1)) + 4096)
    rx = ingest.ShmReceiver("agg", untrack=False)
    try:
        size = snd.send(m1)
        msg = rx.loads(tag, size)
        assert msg["weights"]["w"].is_pinned()       # registered: the kernel can stream it
        finish = consume(msg, rx, tag)
        del msg
        snd.send(m2)                                 # the sender's next message, same segment
        return m1, finish()
    finally:
        rx.close()
        snd.close()


@pytest.mark.oracle
def test_fedbuff_deferred_arrival_survives_segment_rewrite():
    from oracle import oracle as Ora
    opt = S_make("fedbuff")
    state = {}

    def consume(msg, rx, tag):
        c = S.SortedCache()
        c["t0"] = S.TR(msg["weights"], msg["dataset_size"], 5)
        state["agg"] = opt.do(None, c, total=msg["dataset_size"], version=6)   # queued (deferred)
        return lambda: {k: v.cpu() for k, v in state["agg"].items()}          # read after the rewrite
    m1, got = _run(consume)
    exp = Ora.OracleFedBuff().do(None, _one(m1, 5), total=m1["dataset_size"], version=6)
    S.assert_bitwise("fedbuff/shm", got, exp)


@pytest.mark.oracle
def test_fedavg_zero_copy_read_finishes_before_do_returns():
    from oracle import oracle as Ora
    g = torch.Generator().manual_seed(3)
    base = {"w": torch.randn(P, generator=g), "b": torch.randn(37, generator=g)}
    state = {}

    def consume(msg, rx, tag):
        c = S.SortedCache()
        c["t0"] = S.TR(msg["weights"], msg["dataset_size"])
        state["out"] = S_make("fedavg").do(S.to_dev(base, DEV), c, total=msg["dataset_size"] * 3)
        return lambda: S.to_cpu(state["out"])
    m1, got = _run(consume)
    exp = {k: v.clone() for k, v in base.items()}
    Ora.OracleFedAvg().do(exp, _one(m1, 0), total=m1["dataset_size"] * 3)
    S.assert_bitwise("fedavg/shm", got, exp)


@pytest.mark.oracle
@pytest.mark.parametrize("placement", ["slab", "hbm", "host"])
def test_device_update_cache_copy_completes_before_setitem_returns(placement):
    from flame_amd import ingest
    from oracle import oracle as Ora
    g = torch.Generator().manual_seed(4)
    base = {"w": torch.randn(P, generator=g), "b": torch.randn(37, generator=g)}
    cache = ingest.DeviceUpdateCache(device=DEV, placement=placement, capacity=2)

    def consume(msg, rx, tag):
        cache["t0"] = S.TR(msg["weights"], msg["dataset_size"])

        def finish():
            out = S_make("fedavg").do(S.to_dev(base, DEV), cache, total=msg_total)
            return S.to_cpu(out)
        return finish
    msg_total = 10
    m1, got = _run(consume)
    exp = {k: v.clone() for k, v in base.items()}
    Ora.OracleFedAvg().do(exp, _one(m1, 0), total=msg_total)
    S.assert_bitwise(f"cache/{placement}", got, exp)


def test_stale_view_raises_instead_of_reading_torn_data():
    """A view kept in a plain cache past the sender's next message is refused."""
    from flame_amd import ingest
    m1, m2 = _msgs(72)
    tag = f"flamestale{os.getpid()}"
    snd = _Sender(tag, len(cloudpickle.dumps(m1)) + 4096)
    rx = ingest.ShmReceiver("agg", untrack=False)
    try:
        old = rx.loads(tag, snd.send(m1))
        c = S.SortedCache()
        c["t0"] = S.TR(old["weights"], old["dataset_size"])
        new = rx.loads(tag, snd.send(m2))            # the next message arrives through the segment
        with pytest.raises(RuntimeError, match="stale shared-memory view"):
            S_make("fedavg").do({k: torch.zeros_like(v, device=DEV) for k, v in m1["weights"].items()}, c,
                                total=10)
        c2 = S.SortedCache()
        c2["t1"] = S.TR(new["weights"], new["dataset_size"])      # the live message is fine
        S_make("fedavg").do({k: torch.zeros_like(v, device=DEV) for k, v in m1["weights"].items()}, c2, total=11)
        torch.cuda.synchronize()
        del old, new, c, c2
    finally:
        rx.close()
        snd.close()


def _one(msg, version):
    c = S.SortedCache()
    c["t0"] = S.TR({k: v.clone() for k, v in msg["weights"].items()}, msg["dataset_size"], version)
    return c


def S_make(sort, **kw):
    from flame_amd.optimizers import optimizer_provider
    return optimizer_provider.get(sort, **kw)
