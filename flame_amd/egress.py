"""Egress path: the aggregated model back onto flame's channel (the other side of the hot path).

The reference's ``_distribute_weights`` (``mode/horizontal/syncfl/top_aggregator.py:184-215``)
sends, for EVERY selected end, ``{WEIGHTS: weights_to_device(self.weights, CPU), ROUND: r,
DATASAMPLER_METADATA: md}`` through ``channel.send`` (``channel.py:203-218``), i.e. one D2H
copy of the whole model and one ``cloudpickle.dumps`` per end.  ``dumps`` serialises each tensor
through torch's legacy ``torch.save`` into a bytes object that the pickler copies again
(measured 149 ms for a 100 MB model on this container's CPU).  The message is the same for
every end of a round.

:class:`MessageEncoder` builds that payload ONCE: a pickle any ``cloudpickle.loads`` (the
trainer's channel) -- and :func:`flame_amd.ingest.decode` -- reads back as the same message.
Non-tensor parts go through cloudpickle (protocol 3, so arbitrary metadata still works);
every tensor becomes torch's own reduce, ``torch._utils._rebuild_tensor_v2(
torch.storage._load_from_bytes(<legacy torch.save stream>), 0, size, stride, False,
OrderedDict())``, whose stream (torch's header, the storage record, the raw bytes) is written
straight into one pinned output buffer -- a device tensor's bytes by ONE D2H copy into their
final place, no host staging, no second copy.  Tensors are serialised contiguous, with only
their own elements (a view does not drag its whole base storage along, unlike ``dumps``).
"""
from __future__ import annotations

import collections
import io
import os
import pickle
from typing import Any, List

import numpy as np
import torch

from .ingest import LEGACY_MAGIC, _STORAGE_DTYPES

_STORAGE_NAME = {dt: name for name, dt in _STORAGE_DTYPES.items()}
_MARK_LEN = 10                               # random mark (per encode) + 6-byte index: a tensor's placeholder
_HEADER = None                               # torch's legacy stream header (magic, protocol, sys info)


def _legacy_header() -> bytes:
    """The three pickles torch's legacy ``_save`` writes before any storage record (the magic
    number, the protocol version, the sys-info dict) -- taken from torch itself once."""
    global _HEADER
    if _HEADER is None:
        bio = io.BytesIO()
        import warnings
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            torch.save(torch.zeros(1).storage(), bio, _use_new_zipfile_serialization=False)
        s = bio.getvalue()
        i = s.find(b"\x80\x02(X\x07\x00\x00\x00storage")
        magic = b"\x80\x02\x8a\x0a" + LEGACY_MAGIC.to_bytes(10, "little") + b"."
        if i <= 0 or not s.startswith(magic):
            raise RuntimeError("flame_amd.egress: unexpected torch legacy stream layout")
        _HEADER = s[:i]
    return _HEADER


def _pickle_ints(x: int):
    """Protocol-2 encodings of a non-negative int that any unpickler reads as ``x`` (the
    canonical one first): BININT1 / BININT2 / BININT / LONG1 -- their different lengths let the
    stream place a storage's raw bytes on an aligned offset."""
    out = []
    if x <= 0xFF:
        out.append(b"K" + bytes([x]))
    if x <= 0xFFFF:
        out.append(b"M" + x.to_bytes(2, "little"))
    if x < (1 << 31):
        out.append(b"J" + x.to_bytes(4, "little", signed=True))
    n = (x.bit_length() + 8) // 8
    out += [b"\x8a" + bytes([m]) + x.to_bytes(m, "little", signed=True) for m in (n, n + 1)]
    return out


def _unicode(s: str) -> bytes:
    b = s.encode("utf-8")
    return b"X" + len(b).to_bytes(4, "little") + b


def storage_stream_head(dtype: torch.dtype, numel: int, key: str = "0", numel_op: bytes = None) -> bytes:
    """Everything torch's legacy ``_save`` of one CPU storage writes before the raw bytes: the
    header, the storage record ``('storage', torch.<T>Storage, key, 'cpu', numel, None)``
    (persistent id), the key list and the u64 element count."""
    name = _STORAGE_NAME.get(dtype)
    if name is None:
        raise TypeError(f"flame_amd.egress: no legacy storage type for {dtype}")
    rec = (b"\x80\x02(" + _unicode("storage") + b"q\x00" + b"ctorch\n" + name.encode() + b"\nq\x01"
           + _unicode(key) + b"q\x02" + _unicode("cpu") + b"q\x03" + (numel_op or _pickle_ints(numel)[0])
           + b"Ntq\x04Q.")
    keys = b"\x80\x02]q\x00" + _unicode(key) + b"q\x01a."
    return _legacy_header() + rec + keys + numel.to_bytes(8, "little")


def _aligned_head(dtype, numel, nbytes, at: int, align: int = 64):
    """(BINBYTES opcode + storage_stream_head) for a storage whose BINBYTES opcode starts at
    offset ``at``, with the key's length and the element count's encoding chosen so that the raw
    bytes start on an ``align``-byte boundary (the storage key is free text in torch's format)."""
    for L in range(1, align + 2):
        for op in _pickle_ints(numel):
            head = storage_stream_head(dtype, numel, "0" * L, op)
            blen = len(head) + nbytes
            bop = (b"B" + blen.to_bytes(4, "little")) if blen < (1 << 32) else (b"\x8e" + blen.to_bytes(8, "little"))
            if (at + len(bop) + len(head)) % align == 0:
                return bop + head
    raise AssertionError("unreachable: key lengths cover every residue")


class _StoragePlaceholder:
    __slots__ = ("mark",)

    def __init__(self, mark):
        self.mark = mark

    def __reduce__(self):
        return (torch.storage._load_from_bytes, (self.mark,))


def _pickler_base():
    try:
        import cloudpickle
        return cloudpickle.Pickler
    except ImportError:        # pragma: no cover - flame always ships cloudpickle
        return pickle.Pickler


class _SkeletonPickler(_pickler_base()):
    """cloudpickle (protocol 3: no frames) with every tensor replaced by torch's reduce over a
    16-byte placeholder storage; the tensors are collected in pickling order."""

    def __init__(self, f, tensors: List[torch.Tensor], mark: bytes):
        super().__init__(f, protocol=3)
        self._tensors = tensors
        self._mark = mark

    def reducer_override(self, obj):
        if isinstance(obj, torch.Tensor):
            if obj.requires_grad or obj.is_sparse or obj.is_quantized or obj.dtype not in _STORAGE_NAME:
                raise TypeError(f"flame_amd.egress: tensor of {obj.dtype} / layout {obj.layout} is not a model weight")
            i = len(self._tensors)
            self._tensors.append(obj)
            shape = tuple(obj.shape)
            stride, acc = [], 1
            for d in reversed(shape):
                stride.append(acc)
                acc *= d
            return (torch._utils._rebuild_tensor_v2,
                    (_StoragePlaceholder(self._mark + i.to_bytes(6, "little")), 0, shape, tuple(reversed(stride)), False,
                     collections.OrderedDict()))
        sup = getattr(super(), "reducer_override", None)
        return sup(obj) if sup is not None else NotImplemented


def _layout(message: Any, mark: bytes):
    """The payload of ``message`` as ``([(offset, bytes | tensor)], total bytes)``: the pickle's
    own bytes, and each tensor's raw bytes at a 64-byte aligned offset (its storage stream head
    right before it).  A pure function of the message's structure and ``mark``."""
    tensors: List[torch.Tensor] = []
    f = io.BytesIO()
    _SkeletonPickler(f, tensors, mark).dump(message)
    skel = f.getvalue()
    # the placeholders, in order: SHORT_BINBYTES 16 <mark i> -> the storage's whole stream,
    # its raw bytes 64-byte aligned in the payload (so a device tensor lands by one aligned DMA)
    pieces, pos, off = [], 0, 0
    for i, t in enumerate(tensors):
        ph = b"C\x10" + mark + i.to_bytes(6, "little")
        j = skel.find(ph, pos)
        if j < 0:
            raise RuntimeError("flame_amd.egress: placeholder not found in the skeleton")
        pieces.append((off, skel[pos:j]))
        off += j - pos
        nb = t.numel() * t.element_size()
        head = _aligned_head(t.dtype, t.numel(), nb, off)
        pieces.append((off, head))
        off += len(head)
        pieces.append((off, t))
        off += nb
        pos = j + len(ph)
    pieces.append((off, skel[pos:]))
    return pieces, off + len(skel) - pos


class MessageEncoder:
    """Encodes flame messages whose tensors (device or host) go straight into one pinned payload
    buffer.  ``encode`` returns a read-only ``memoryview`` of that buffer, valid until the next
    ``encode`` on this encoder reuses it (``ring`` buffers are cycled; each is reused only once
    the copies into it have completed); ``encode_bytes`` returns an independent ``bytes``."""

    def __init__(self, ring: int = 2, pin: bool = True):
        self.ring = max(1, int(ring))
        self.pin = pin and torch.cuda.is_available()
        self._bufs = [None] * self.ring
        self._next = 0

    def _buffer(self, nbytes):
        i = self._next
        self._next = (i + 1) % self.ring
        buf = self._bufs[i]
        if buf is None or buf.numel() < nbytes:
            buf = torch.empty(max(nbytes, 1 << 20), dtype=torch.uint8, pin_memory=self.pin)
            self._bufs[i] = buf
        return buf

    def encode(self, message: Any) -> memoryview:
        # a fresh random mark per message: no bytes of the message itself can pass for a placeholder
        pieces, total = _layout(message, os.urandom(_MARK_LEN))
        buf = self._buffer(total)
        out = buf.numpy()
        copies = set()          # devices whose streams carry D2H copies into the buffer
        for off, pc in pieces:
            if isinstance(pc, bytes):
                out[off:off + len(pc)] = np.frombuffer(pc, dtype=np.uint8)
                continue
            nb = pc.numel() * pc.element_size()
            if nb:
                dst = buf[off:off + nb].view(pc.dtype).view(pc.shape if pc.dim() else ())
                src = pc.detach()
                if src.is_cuda:
                    dst.copy_(src, non_blocking=True)      # D2H straight into the payload
                    copies.add(src.device)
                else:
                    dst.copy_(src)
        for d in copies:        # the payload is complete when encode returns
            torch.cuda.current_stream(d).synchronize()
        return memoryview(out[:total]).toreadonly()

    def encode_bytes(self, message: Any) -> bytes:
        return bytes(self.encode(message))


_default = None


def dumps(message: Any) -> bytes:
    """One-shot :meth:`MessageEncoder.encode_bytes` (a ``cloudpickle.dumps`` stand-in for
    weight messages: ``cloudpickle.loads`` returns an equal message)."""
    global _default
    if _default is None:
        _default = MessageEncoder(ring=1, pin=os.environ.get("FLAME_AMD_EGRESS_PIN", "1") != "0")
    return _default.encode_bytes(message)


class ShardedEgress:
    """The model message of a parameter-sharded aggregator, written into ONE host payload by every
    rank at once (the other side of ``DeviceUpdateCache(shard=plan)``'s ingest).

    Each rank D2Hs only ITS ranges of the model -- the plan's owned pieces of every key; rank 0 also
    the replicated key tails and the pickle's own bytes -- over its own PCIe link, straight into a
    POSIX shared-memory segment that every rank has mapped and page-locked; after a barrier rank 0
    holds the complete payload (``encode`` returns it there, ``None`` elsewhere), byte-for-byte what
    :class:`MessageEncoder` builds.  With ``ShardedOptimizer(gather=False)`` the model never crosses
    xGMI: at N GPUs the egress is N links' D2H of 1/N of the model each instead of one link's D2H of
    all of it behind an all-gather (``syncfl/top_aggregator.py:184-215`` sends the model from host
    memory anyway).

    ``message`` must be the same structure on every rank; tensors that are values of
    ``message["weights"]`` under the plan's keys are written by range, any other tensor whole by
    rank 0.  The placeholder mark is drawn from a seed rank 0 broadcasts once (every rank builds the
    same layout without exchanging it per message)."""

    def __init__(self, plan, name: str, group=None):
        import torch.distributed as dist
        self.plan, self.name, self.group = plan, name, group
        self.dist = dist if (dist.is_available() and dist.is_initialized()) else None
        self.rank = self.dist.get_rank(group) if self.dist else 0
        self.world = self.dist.get_world_size(group) if self.dist else 1
        seed = [os.urandom(16) if self.rank == 0 else None]
        if self.dist and self.world > 1:
            src = dist.get_global_rank(group, 0) if group is not None else 0
            self.dist.broadcast_object_list(seed, src=src, group=group)
        self._seed, self._seq = seed[0], 0
        self._seg = self._reg = None
        self._size = 0

    def _barrier(self):
        if self.dist and self.world > 1:
            self.dist.barrier(group=self.group)

    def _segment(self, total: int) -> None:
        if self._seg is not None and self._size >= total:
            return
        self.close()
        from multiprocessing import shared_memory
        from .ingest import RegisteredBuffer
        size = -(-max(total, 1) // (1 << 20)) * (1 << 20)
        nm = f"{self.name}-{size}"
        seg = None
        if self.rank == 0:
            try:                                  # a stale segment of a crashed run
                old = shared_memory.SharedMemory(nm)
                old.close()
                old.unlink()
            except FileNotFoundError:
                pass
            seg = shared_memory.SharedMemory(nm, create=True, size=size)
        self._barrier()
        if seg is None:
            seg = shared_memory.SharedMemory(nm)
            try:                                  # rank 0 owns (and unlinks) the segment
                from multiprocessing import resource_tracker
                resource_tracker.unregister(seg._name, "shared_memory")  # noqa: SLF001
            except Exception:  # noqa: BLE001
                pass
        self._reg = RegisteredBuffer(seg.buf) if torch.cuda.is_available() else None
        self._seg, self._size = seg, size

    def encode(self, message: Any):
        import hashlib
        self._seq += 1
        mark = hashlib.blake2b(self._seed + self._seq.to_bytes(8, "little"), digest_size=_MARK_LEN).digest()
        pieces, total = _layout(message, mark)
        self._segment(total)
        buf = torch.frombuffer(self._seg.buf, dtype=torch.uint8)
        out = buf.numpy()
        weights = message.get("weights") if isinstance(message, dict) else None
        by_id = {id(v): k for k, v in weights.items() if k in self.plan.numel} if isinstance(weights, dict) else {}
        devices = set()

        def put(off, src):
            nb = src.numel() * src.element_size()
            if nb:
                dst = buf[off:off + nb].view(src.dtype)
                dst.copy_(src.reshape(-1), non_blocking=src.is_cuda)
                if src.is_cuda:
                    devices.add(src.device)
        for off, pc in pieces:
            if isinstance(pc, bytes):
                if self.rank == 0:
                    out[off:off + len(pc)] = np.frombuffer(pc, dtype=np.uint8)
                continue
            key = by_id.get(id(pc))
            flat = pc.detach().reshape(-1)
            if key is None:
                if self.rank == 0:
                    put(off, flat)
                continue
            s = flat.element_size()
            for sub in self.plan.subs:
                if sub.key == key and sub.hi > sub.lo and (not sub.tail or self.rank == 0):
                    put(off + sub.lo * s, flat[sub.lo:sub.hi])
        for d in devices:
            torch.cuda.current_stream(d).synchronize()
        self._barrier()                           # every rank's ranges are in the payload
        if self.rank != 0:
            return None
        return memoryview(out[:total]).toreadonly()

    def close(self) -> None:
        if self._seg is None:
            return
        if self._reg is not None:
            self._reg.close()
        self._reg = None
        seg, self._seg, self._size = self._seg, None, 0
        self._barrier()                           # nobody maps it any more
        try:
            seg.close()
        except BufferError:
            pass
        if self.rank == 0:
            try:
                seg.unlink()
            except FileNotFoundError:
                pass
