"""Lifetime of zero-copy views into senders' shared-memory segments.

The LIFL SHM backend's sender rewrites its segment for its next message
(``backend/shm.py:393-403``); the reference receiver therefore copies every message
out of the segment on arrival (``:386-391``).  :class:`flame_amd.ingest.ShmReceiver`
instead decodes in place, so every consumer that could outlive the call that handed
it a view must either finish reading the segment before returning or copy the data
out first.  This module is the registry they consult:

* the address ranges of the segments a receiver has open (``add`` / ``remove``,
  ``aliases(t)``: does a host tensor point into one?), and
* each segment's message generation, stamped on the tensors a message was decoded
  into (``stamp``); ``check_live(t)`` raises if the sender has since delivered a newer
  message through the same segment (the view's bytes are gone).

The consumers (engine, FedBuff's deferred aggregate, DeviceUpdateCache) act on it:
a kernel streaming a segment zero-copy is waited for before the launching call
returns, a deferred FedBuff arrival and a cache entry are copied to HBM before the
call returns -- the reference's "copy on receive" guarantee, with the copy done by
the DMA engine straight into HBM instead of a host memcpy + unpickle.
"""
from __future__ import annotations

import bisect
import threading

_lock = threading.Lock()
_starts = []          # sorted segment start addresses
_ranges = {}          # start -> (end, name)
_by_name = {}         # name -> start
_gen = {}             # name -> generation of the segment's current message


def add(name: str, start: int, nbytes: int) -> None:
    with _lock:
        if name in _by_name:
            _remove_locked(name)
        bisect.insort(_starts, start)
        _ranges[start] = (start + nbytes, name)
        _by_name[name] = start
        _gen.setdefault(name, 0)


def _remove_locked(name: str) -> None:
    start = _by_name.pop(name, None)
    if start is not None:
        _ranges.pop(start, None)
        i = bisect.bisect_left(_starts, start)
        if i < len(_starts) and _starts[i] == start:
            _starts.pop(i)


def remove(name: str) -> None:
    with _lock:
        _remove_locked(name)


def active() -> bool:
    """Is any shared-memory segment open (could any host tensor alias one)?"""
    return bool(_starts)


def segment_of(ptr: int):
    """Name of the open segment containing host address ``ptr`` (or None)."""
    if not _starts:
        return None
    i = bisect.bisect_right(_starts, ptr) - 1
    if i < 0:
        return None
    end, name = _ranges[_starts[i]]
    return name if ptr < end else None


def aliases(t) -> bool:
    """Does host tensor ``t`` read bytes of an open shared-memory segment?"""
    if not _starts or getattr(t, "is_cuda", True) or t.numel() == 0:
        return False
    return segment_of(t.data_ptr()) is not None


def next_generation(name: str) -> int:
    """A new message arrived through segment ``name``: views of older messages are stale."""
    with _lock:
        _gen[name] = _gen.get(name, 0) + 1
        return _gen[name]


def stamp(obj, name: str, gen: int):
    """Mark every tensor in a decoded message (dicts / lists / tuples) as generation ``gen``
    of segment ``name``."""
    import torch
    stack = [obj]
    while stack:
        o = stack.pop()
        if isinstance(o, torch.Tensor):
            o._flame_shm = (name, gen)
        elif isinstance(o, dict):
            stack.extend(o.values())
        elif isinstance(o, (list, tuple)):
            stack.extend(o)
    return obj


def check_live(t) -> None:
    """Raise if ``t`` was decoded from a segment that has since carried a newer message."""
    tag = getattr(t, "_flame_shm", None)
    if tag is not None and _gen.get(tag[0]) != tag[1]:
        raise RuntimeError(f"flame_amd: stale shared-memory view -- sender segment {tag[0]!r} now holds message "
                           f"{_gen.get(tag[0])}, this tensor belongs to message {tag[1]}; a consumer held the view "
                           f"past the sender's next write (copy it out, or aggregate before replying)")
