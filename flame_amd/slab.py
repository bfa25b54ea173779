"""Tiled, device-resident update store (the HBM layout of the MI355X path).

Why tiled.  With one allocation per client update, a workgroup of the
reduction reads one 4 KiB piece from each of N client rows that lie ~P·s bytes
apart, so the ~2,000 resident workgroups keep tens of thousands of distinct
pages in flight; with the updates stored as ``[tiles][N][T]`` (T = one kernel
chunk) a workgroup streams ONE contiguous N·T·s region.  Measured on MI355X
(tools/kernel_sweep.py, same process, 1024 × 25M fp32): 15.78 ms row layout vs
15.10 ms tiled = the plain streaming-read probe (15.13 ms), i.e. +4.5 %.

Layout.  Per dtype group of the model template, every key occupies
``ceil(numel / T)`` whole tiles (keys start on tile boundaries; the padding is
< T elements per key per client), and tile ``t`` holds
``[capacity][T]`` -- slot ``i``'s chunk at ``((t * capacity) + i) * T``.  A slot's
tensor for key ``k`` is exposed as a strided torch view of shape
``(tiles_k, T)`` with strides ``(capacity * T, 1)``; the engine recognises such
views and passes ``client_tile_stride = capacity * T * itemsize`` to the kernel
(``include/flame_amd.h``).  Elements past ``numel`` in a key's last tile are
never read.

Slots are reused stream-ordered: a slot is returned to the free list when the
``SlotWeights`` dict handed out for it is garbage-collected (after the launch
that consumed it), with an event recorded on the then-current stream; the next
write into the slot waits for that event.
"""
from __future__ import annotations

import collections
import collections.abc
import os
from typing import Dict, List

import numpy as np
import torch

from . import _native as N
from . import engine


# pageable payload spans of at least this many bytes are staged through pinned memory
PINNED_STAGE_MIN = 256 << 10
PINNED_RING = 4
# a payload span is staged as one transfer only if it is at most this much larger than the
# tensor bytes it carries (pickle framing and storage headers are a few hundred bytes per key)
STAGE_SPAN_SLACK = 1.25
# a page-locked host source that is not 4-byte aligned (hipMemcpy2DAsync runs ~5 GB/s there):
# "stage" = a contiguous DMA into HBM + the tile kernel, "mapped" = the tile kernel reading it over
# PCIe through its device-mapped address (tools/ingest_diag.py measures both)
MISALIGNED_HOST = os.environ.get("FLAME_AMD_MISALIGNED_HOST", "stage")


class SlotWeights(dict):
    """The weights dict of one slab slot: {key: tiled view}; ``shapes`` holds the model
    shapes; releases the slot when dropped."""

    __slots__ = ("__weakref__", "_release", "shapes", "slab", "slot")

    def __del__(self):
        rel = getattr(self, "_release", None)
        if rel is not None:
            self._release = None
            try:
                rel()
            except Exception:  # noqa: BLE001  (interpreter shutdown)
                pass


class MixedSlotWeights(dict):
    """An update whose kernel-dtype keys sit in a slab slot (tiled views) and whose bool /
    uint8 / int8 / int16 buffers are plain device tensors beside it, in the update's key
    order.  No ``slab`` attribute: the engine takes the generic path, reading the tiled
    views tiled (``client_tile_stride``); ``shapes`` gives every key's model shape; holds
    the slot's :class:`SlotWeights` so the slot is not recycled while this is alive."""

    __slots__ = ("__weakref__", "shapes", "_owner")

    @classmethod
    def of(cls, slot: "SlotWeights", extra, order) -> "MixedSlotWeights":
        w = cls((k, slot[k] if k in slot else extra[k]) for k in order)
        w.shapes = {k: (slot.shapes[k] if k in slot else tuple(extra[k].shape)) for k in order}
        w._owner = slot
        return w


class SlabRef(collections.abc.Mapping):
    """Named element ranges of ONE slab slot: ``{name: (slab_key, lo, hi)}`` -- e.g. this
    rank's slices of a client update (flame_amd.shard).  Tiled views are made only when a
    value is read; the engine computes pointer rows from ``slab`` / ``slot`` / ``ranges``
    without touching them.  ``lo`` must start a slab tile.  Holds the slot's
    :class:`SlotWeights` (``owner``) so the slot is not recycled while this is alive."""

    __slots__ = ("slab", "slot", "ranges", "shapes", "_owner")

    def __init__(self, slab: "UpdateSlab", slot: int, ranges, shapes, owner=None):
        self.slab, self.slot, self.ranges, self.shapes, self._owner = slab, slot, ranges, shapes, owner

    def __getitem__(self, name):
        key, lo, hi = self.ranges[name]
        v = self.slab.slot_view(self.slot, key)
        T = v.shape[1]
        return v[lo // T: max(lo // T + 1, -(-hi // T))]

    def __iter__(self):
        return iter(self.ranges)

    def __len__(self):
        return len(self.ranges)

    def __contains__(self, name):
        return name in self.ranges


class UpdateSlab:
    """``capacity`` client updates shaped like ``template``, tiled in HBM."""

    def __init__(self, template: Dict[str, torch.Tensor], capacity: int, device=None):
        self.device = torch.device(device) if device is not None else engine.pick_device(template)
        self.capacity = int(capacity)
        self.keys: List[str] = list(template.keys())
        self.meta = {}           # key -> (dtype, shape, numel, tile0, tiles)
        tiles_per_dtype = collections.OrderedDict()
        for k in self.keys:
            t = template[k]
            code = engine.dtype_code(t.dtype)
            T = engine.chunk_elems(code)
            tiles = max(1, -(-t.numel() // T))
            tile0 = tiles_per_dtype.get(t.dtype, 0)
            tiles_per_dtype[t.dtype] = tile0 + tiles
            self.meta[k] = (t.dtype, tuple(t.shape), t.numel(), tile0, tiles)
        self.storage = {}        # dtype -> tensor [tiles][capacity][T]
        for dt, tiles in tiles_per_dtype.items():
            T = engine.chunk_elems(engine.dtype_code(dt))
            self.storage[dt] = torch.empty((tiles, self.capacity, T), dtype=dt, device=self.device)
        self._free = collections.deque(range(self.capacity))
        self._ready = {}         # slot -> event the next writer must wait for
        self._stream = None
        self._wt = None          # per-key insert table (see _write_table)
        self._slot_views = {}    # slot -> [(key, tiled view)] (see views)
        self._ring_bufs = [None] * PINNED_RING      # pinned staging of pageable payloads (_pinned_stage)
        self._ring_events = [None] * PINNED_RING
        self._ring_next = 0

    # ------------------------------------------------------------------ slots
    def nbytes(self) -> int:
        return sum(s.numel() * s.element_size() for s in self.storage.values())

    def acquire(self) -> int:
        if not self._free:
            raise RuntimeError(f"UpdateSlab full ({self.capacity} slots); raise capacity")
        return self._free.popleft()

    def _release(self, slot: int) -> None:
        if torch.cuda.is_available():
            ev = torch.cuda.Event()
            ev.record(engine.current_stream(self.device))
            self._ready[slot] = ev
        self._free.append(slot)

    def views(self, slot: int) -> SlotWeights:
        """Tiled views of ``slot`` (what the optimizers receive as ``TrainResult.weights``).
        A slot's view tensors are made once and shared by every SlotWeights of that slot (the
        storage never moves; only the dict and its release hook are per insert)."""
        cached = self._slot_views.get(slot)
        if cached is None:
            cached = self._slot_views[slot] = [(k, self.slot_view(slot, k)) for k in self.keys]
        w = SlotWeights(cached)
        w._release = lambda s=slot: self._release(s)
        w.shapes = {k: self.meta[k][1] for k in self.keys}
        w.slab, w.slot = self, slot     # lets the engine compute pointer rows without touching views
        return w

    def key_layout(self, key: str):
        """(dtype, numel, address of slot 0's first tile, bytes between slots, bytes between tiles)."""
        dt, _, n, tile0, _ = self.meta[key]
        st = self.storage[dt]
        T = st.shape[2]
        isz = st.element_size()
        return dt, n, st.data_ptr() + tile0 * self.capacity * T * isz, T * isz, self.capacity * T * isz

    def slot_view(self, slot: int, key: str) -> torch.Tensor:
        dt, _, _, tile0, tiles = self.meta[key]
        return self.storage[dt][tile0:tile0 + tiles, slot, :]

    # ------------------------------------------------------------------ writes
    def _write_table(self):
        """Per key: (address of slot 0's first tile, bytes, tile stride) -- the slot-independent
        part of a flame_tile_copy row (``include/flame_amd.h``)."""
        if self._wt is None:
            rows = []
            for k in self.keys:
                dt, n, base, slot_bytes, tile_stride = self.key_layout(k)
                if slot_bytes != N.FLAME_TILE_BYTES:
                    raise AssertionError(f"slab tile of {k} is {slot_bytes} B, the insert kernel copies "
                                         f"{N.FLAME_TILE_BYTES} B tiles")
                rows.append((base, n * self.storage[dt].element_size(), tile_stride))
            self._wt = np.asarray(rows, dtype=np.int64).reshape(-1, 3)
        return self._wt

    def write(self, slot: int, weights: Dict[str, torch.Tensor], stream=None) -> None:
        """Copy one client's update (host or device tensors) into ``slot`` on ``stream``.

        Device sources: ONE ``flame_slab_write`` launch tiles every key into the slot (the
        table rides in the kernel arguments).  Host tensors that are views into one decoded
        channel payload (``ingest.decode``): the payload span holding them crosses PCIe in ONE
        transfer and joins that launch (:meth:`_stage_payloads`).  Other host sources (pinned,
        registered or pageable): ``flame_slab_write_2d``, one pitched copy-engine transfer per
        key, no staging tensor.
        """
        cur = engine.current_stream(self.device)
        st = stream or cur
        for k in self.keys:     # validate before the slot's reader event is consumed (a refused
            if k not in weights:    # write leaves the slot guarded for the next writer)
                raise KeyError(k)
            dt, _, n, _, _ = self.meta[k]
            src = weights[k]
            if src.numel() != n:
                raise RuntimeError(f"{k}: {src.numel()} elements, slab expects {n}")
            if src.dtype != dt:
                raise NotImplementedError(f"{k}: dtype {src.dtype} != slab dtype {dt}")
        ev = self._ready.pop(slot, None)
        if ev is not None:
            st.wait_event(ev)
        wt = self._write_table()
        dev_rows, host_rows, keep = [], [], []
        sync = False
        for i, k in enumerate(self.keys):
            dt, shape, n, tile0, tiles = self.meta[k]
            src = weights[k]
            if src.is_cuda and src.device != self.device:
                with torch.cuda.stream(st):
                    src = src.to(self.device, non_blocking=True)
            if not src.is_contiguous():
                if src.is_cuda:
                    with torch.cuda.stream(st):
                        src = src.contiguous()
                else:
                    src = src.contiguous()
                    sync = True        # a host temporary: the copy must finish before it is freed
            if n == 0:
                continue
            row = (src.data_ptr(), int(wt[i, 0]) + slot * N.FLAME_TILE_BYTES, int(wt[i, 1]), int(wt[i, 2]))
            if src.is_cuda:
                dev_rows.append(row)
                keep.append(src)
            else:
                host_rows.append(row)
                keep.append(src)
        staged = []
        if len(host_rows) > 1:
            dev_rows += self._stage_payloads(host_rows, keep, st, staged)
        # hipMemcpy2DAsync drops to ~5 GB/s for a host source that is not 4-byte aligned -- and a
        # storage inside a pickled payload starts anywhere (a decoded view into a LIFL shm segment,
        # or this rank's slice of one) -- against ~50 GB/s for the tile-copy kernel reading the same
        # page-locked bytes over PCIe through their device-mapped address
        # (profiles/r06e2_h2d_paths.log, r06e_ingest_diag.log)
        mapped = []
        if host_rows:
            by_src = {(t.data_ptr(), t.numel() * t.element_size()): t for t in keep if not t.is_cuda}
            for r in [r for r in host_rows if r[0] % 4]:
                t = by_src.get((r[0], r[2]))       # the row's source: same address, same bytes
                if t is None or not t.is_pinned():
                    continue
                host_rows.remove(r)
                if MISALIGNED_HOST == "mapped":
                    dev_rows.append((engine.host_device_pointer(r[0]), r[1], r[2], r[3]))
                    mapped.append(t)
                else:        # "stage": one contiguous DMA (full rate at any alignment), then the kernel tiles it in HBM
                    with torch.cuda.stream(st):
                        d = t.reshape(-1).to(self.device, non_blocking=True)
                    d.record_stream(st)
                    keep.append(d)
                    staged.append(t)
                    dev_rows.append((d.data_ptr(), r[1], r[2], r[3]))
        L = N.lib()
        if dev_rows:
            tab = np.asarray(dev_rows, dtype=np.uint64).view(np.int64)
            N.check(L.flame_slab_write(tab.ctypes.data, len(dev_rows), st.cuda_stream))
            if st != cur:
                for t in keep:
                    if t.is_cuda:
                        t.record_stream(st)       # read on `st`: keep the caching allocator off it
            if staged:
                engine._staging.hold_on(st, staged)
            if mapped:       # read by the kernel over PCIe: held until it has run
                engine._staging.hold_on(st, mapped)
        if host_rows:
            tab = np.asarray(host_rows, dtype=np.uint64).view(np.int64)
            N.check(L.flame_slab_write_2d(tab.ctypes.data, len(host_rows), st.cuda_stream))
            if sync:
                st.synchronize()
            else:       # the copy engine reads the host tensors after this returns: hold them
                engine._staging.hold_on(st, [t for t in keep if not t.is_cuda])

    def write_key(self, slot: int, key: str, src: torch.Tensor) -> None:
        """Copy one key of ``slot`` from a device tensor (one ``flame_slab_write`` launch on the
        current stream); the rest of the slot is untouched."""
        dt, _, n, _, _ = self.meta[key]
        if src.numel() != n or src.dtype != dt or not src.is_cuda:
            raise ValueError(f"{key}: need a device {dt} tensor of {n} elements")
        if n == 0:
            return
        src = src.contiguous()
        i = self.keys.index(key)
        wt = self._write_table()
        tab = np.asarray([(src.data_ptr(), int(wt[i, 0]) + slot * N.FLAME_TILE_BYTES, int(wt[i, 1]), int(wt[i, 2]))],
                         dtype=np.uint64).view(np.int64)
        N.check(N.lib().flame_slab_write(tab.ctypes.data, 1, engine._stream_ptr(self.device)))

    def _stage_payloads(self, host_rows, keep, st, staged):
        """Host rows whose tensors are views into ONE decoded channel payload
        (``ingest.decode`` tags them with it): the payload's byte span holding them goes to
        the device in ONE transfer, and those rows become device rows reading it (misaligned
        sources are fine for ``flame_slab_write``).  Removes them from ``host_rows``; the host
        spans copied go to ``staged`` (held until the copy has run: a pinned payload's copy is
        asynchronous)."""
        groups = collections.defaultdict(list)
        for src in keep:
            buf = getattr(src, "_flame_payload", None) if not src.is_cuda else None
            if buf is not None:
                groups[id(buf)].append((buf, src.data_ptr(), src.numel() * src.element_size()))
        out = []
        for items in groups.values():
            if len(items) < 2:
                continue
            buf = items[0][0]
            whole = torch.frombuffer(buf, dtype=torch.uint8)        # zero-copy: the payload's address range
            base, end = whole.data_ptr(), whole.data_ptr() + whole.numel()
            lo = min(p for _, p, _ in items)
            hi = max(p + n for _, p, n in items)
            if lo < base or hi > end or hi - lo > STAGE_SPAN_SLACK * sum(n for _, _, n in items) + (64 << 10):
                continue      # outside the buffer, or mostly other bytes (e.g. a big non-weight blob)
            span = whole[lo - base:hi - base]
            ring_slot = None
            if not span.is_pinned() and span.numel() >= PINNED_STAGE_MIN:
                # pageable payload: torch's multi-threaded host copy into a pinned ring slot,
                # then an ASYNCHRONOUS DMA (a pageable H2D blocks the caller for its duration)
                span, ring_slot = self._pinned_stage(span)
            with torch.cuda.stream(st):
                dev = span.to(self.device, non_blocking=True)
            dev.record_stream(st)
            if ring_slot is not None:             # the ring slot is free again once this DMA has run
                self._ring_events[ring_slot] = torch.cuda.Event()
                self._ring_events[ring_slot].record(st)
            keep.append(dev)
            staged.append(whole)
            ptrs = {p for _, p, _ in items}
            moved = [r for r in host_rows if r[0] in ptrs]
            for r in moved:
                host_rows.remove(r)
                out.append((dev.data_ptr() + (r[0] - lo), r[1], r[2], r[3]))
        return out

    def _pinned_stage(self, span: torch.Tensor):
        """``span`` copied into a pinned host buffer: (the copy, its ring slot).  The ring holds
        PINNED_RING buffers per slab; a slot is reused once the DMA that read it has run (the
        caller records ``_ring_events[slot]`` behind that transfer)."""
        i = self._ring_next
        self._ring_next = (i + 1) % PINNED_RING
        ev = self._ring_events[i]
        if ev is not None:
            ev.synchronize()
        buf = self._ring_bufs[i]
        if buf is None or buf.numel() < span.numel():
            buf = self._ring_bufs[i] = torch.empty(max(span.numel(), 1 << 20), dtype=torch.uint8, pin_memory=True)
        out = buf[:span.numel()]
        out.copy_(span)
        return out, i

    def put(self, weights: Dict[str, torch.Tensor], stream=None) -> SlotWeights:
        """Acquire a slot, write ``weights`` into it, return its tiled views."""
        slot = self.acquire()
        try:
            self.write(slot, weights, stream)
        except Exception:
            self._free.appendleft(slot)
            raise
        return self.views(slot)

    def read(self, slot: int, key: str) -> torch.Tensor:
        """A contiguous copy of ``slot``'s tensor ``key`` in its original shape (for inspection)."""
        dt, shape, n, _, _ = self.meta[key]
        return self.slot_view(slot, key).reshape(-1)[:n].reshape(shape).clone()
