"""Host side of the drop-in path: turns state_dict tensors into segment tables
and launches the native kernels (``include/flame_amd.h``) on torch's current stream.

Pure-Python planning (``plan``, ``rate32``, ``chunk_elems``) needs no GPU and is
unit-tested on CPU; the launchers (``reduce_``, ``fedopt_reduce_adapt_``,
``scale_add_``, ``synth_fill_``) need the native library and a HIP device.

A *segment* is one contiguous tensor (one state_dict entry).  For a reduction,
row ``s`` of the client table holds, in cache.iterkeys() order, the device
address of every client's tensor for segment ``s``.  One launch covers all
segments of one dtype, so a whole model aggregates in one kernel per dtype.
"""
from __future__ import annotations

import collections
import ctypes
import os
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np
import torch

from . import _native as N
from . import shm_lease

DTYPE_CODE = {
    torch.float32: N.FLAME_F32, torch.bfloat16: N.FLAME_BF16, torch.float16: N.FLAME_F16,
    torch.float64: N.FLAME_F64, torch.int64: N.FLAME_I64, torch.int32: N.FLAME_I32,
}
FLOAT_CODES = (N.FLAME_F32, N.FLAME_BF16, N.FLAME_F16, N.FLAME_F64)
# state_dict dtypes the kernels do not carry (bool masks, uint8 / int8 / int16 buffers): their
# tmp is formed in fp32 by the kernel and cast, their adds are torch's (see tmp_of)
NARROW = (torch.bool, torch.uint8, torch.int8, torch.int16)
VEC_BYTES = 16
ITEMSIZE = {N.FLAME_F32: 4, N.FLAME_BF16: 2, N.FLAME_F16: 2, N.FLAME_F64: 8, N.FLAME_I64: 8, N.FLAME_I32: 4}


def dtype_code(dt: torch.dtype) -> int:
    try:
        return DTYPE_CODE[dt]
    except KeyError:
        raise TypeError(f"flame_amd: tensor dtype {dt} is not supported by the aggregation kernels "
                        f"(supported: {sorted(str(d) for d in DTYPE_CODE)})") from None


_CHUNK = {}


def chunk_elems(code: int, scale_add: bool = False) -> int:
    """Elements one workgroup covers per chunk, as compiled into the library
    (flame_chunk_elems / flame_scale_add_chunk_elems; the library loads without a GPU)."""
    key = (code, scale_add)
    if key not in _CHUNK:
        L = N.lib()
        _CHUNK[key] = int(L.flame_scale_add_chunk_elems(code) if scale_add else L.flame_chunk_elems(code))
        if _CHUNK[key] <= 0:
            raise TypeError(f"flame_amd: dtype code {code} not supported by this kernel")
    return _CHUNK[key]


def rate32(rate: float) -> float:
    """torch wraps a Python float scalar and rounds it to the fp32 opmath type (RNE)."""
    return float(np.float32(rate))


# ------------------------------------------------------------------ planning (host only)
SEG_WORDS = 10  # int64 words per flame_segment


@dataclass
class Seg:
    numel: int
    out: int = 0
    inp: int = 0
    cur: int = 0
    cur_out: int = 0
    m: int = 0
    v: int = 0
    clients: List[int] = field(default_factory=list)
    tile_stride: int = 0   # bytes between consecutive chunks of one client (0 = contiguous)
    flags: int = 0         # FLAME_SEG_* bits set by the caller (FLAME_SEG_UNALIGNED is computed)

    def pointers(self):
        return [self.out, self.inp, self.cur, self.cur_out, self.m, self.v, self.tile_stride] + list(self.clients)


@dataclass
class Plan:
    code: int
    meta: np.ndarray      # int64 words: [segments (10 each)] [client table] [rates32 | rates64]
    n_segs: int
    n_chunks: int
    n_clients: int
    off_clients: int      # byte offsets into the device copy of ``meta``
    off_r32: int
    off_r64: int


def plan(code: int, segs: Sequence[Seg], rates: Sequence, chunk: Optional[int] = None,
         seg_rates: bool = False, compact: bool = False) -> Plan:
    """Build the device metadata block for one launch (no GPU needed).

    ``rates`` holds one rate per client, or with ``seg_rates`` one row of rates per
    segment (FLAME_AGG_SEG_RATES).  ``compact`` keeps only the rate array the dtype
    reads (its other offset is -1) -- the kernel-argument launch path."""
    n_segs = len(segs)
    if n_segs == 0:
        raise ValueError("empty segment list")
    if seg_rates:
        if len(rates) != n_segs or len({len(r) for r in rates}) > 1:
            raise ValueError("seg_rates: one equal-length rate row per segment")
        n = len(rates[0])
        rates = [r for row in rates for r in row]
    else:
        n = len(rates)
    chunk = chunk or chunk_elems(code)
    head = np.zeros((n_segs, SEG_WORDS), dtype=np.uint64)
    table = np.empty((n_segs, n), dtype=np.uint64)
    begin = 0
    for i, s in enumerate(segs):
        if len(s.clients) != n:
            raise ValueError("every segment needs one pointer per client")
        row = table[i]
        row[:] = s.clients
        fixed = (s.out, s.inp, s.cur, s.cur_out, s.m, s.v)
        unaligned = bool(np.any(row % VEC_BYTES)) or any(p % VEC_BYTES for p in fixed if p)
        head[i] = (*fixed, s.numel, begin, s.flags | (N.FLAME_SEG_UNALIGNED if unaligned else 0), s.tile_stride)
        begin += -(-s.numel // chunk) if s.numel > 0 else 0
    if begin == 0:
        begin = 1  # all segments empty: one (idle) chunk keeps the launch valid
    off_clients = head.size * 8
    off_r32 = off_clients + table.size * 8
    r64 = np.asarray(rates, dtype=np.float64).reshape(-1)
    r32 = r64.astype(np.float32)            # RNE, as torch rounds a Python float scalar
    if r32.size % 2:
        r32 = np.concatenate([r32, np.zeros(1, np.float32)])
    parts = [head.view(np.int64).reshape(-1), table.view(np.int64).reshape(-1)]
    if compact:    # only the rate array the dtype reads (f64 tensors use the fp64 rates)
        if code == N.FLAME_F64:
            off_r64, off_r32 = off_r32, -1
            parts.append(r64.view(np.int64))
        else:
            off_r64 = -1
            parts.append(r32.view(np.int64))
    else:
        off_r64 = off_r32 + r32.size * 4
        parts += [r32.view(np.int64), r64.view(np.int64)]
    return Plan(code, np.concatenate(parts), n_segs, begin, n, off_clients, off_r32, off_r64)


# ------------------------------------------------------------------ device staging
class _Staging:
    """Pinned host -> device upload of plan metadata, ordered on the current stream."""

    def __init__(self):
        self._inflight = collections.deque()
        self._streams = {}

    def upload(self, meta: np.ndarray, device: torch.device) -> torch.Tensor:
        """The copy runs on a side stream, so it overlaps whatever kernel the launch stream is
        still running (the next launch only waits for its own few-KB table, not for a copy
        queued behind the previous kernel); the launch stream waits on the copy's event."""
        while self._inflight and self._inflight[0][0].query():
            self._inflight.popleft()
        host = torch.from_numpy(meta)
        try:
            host = host.pin_memory()
        except RuntimeError:
            pass
        cur = current_stream(device)
        side = self._streams.get(device)
        if side is None:
            side = self._streams[device] = torch.cuda.Stream(device)
        with torch.cuda.stream(side):
            dev = host.to(device, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(side)
        cur.wait_event(ev)
        dev.record_stream(cur)      # allocated on the side stream, read by kernels on the launch stream
        self._inflight.append((ev, host))
        return dev

    def drain(self) -> None:
        """Wait for every in-flight staging copy / zero-copy read and drop the host refs."""
        while self._inflight:
            ev, _ = self._inflight.popleft()
            ev.synchronize()

    def hold_on(self, stream, host_tensors) -> None:
        """Keep host tensors an asynchronous copy on ``stream`` reads alive until it has passed
        this point (a view of a sender's shared-memory segment: wait here, see ``hold``)."""
        ev = torch.cuda.Event()
        ev.record(stream)
        if any(shm_lease.aliases(t) for t in host_tensors):
            ev.synchronize()
            return
        self._inflight.append((ev, list(host_tensors)))

    def hold(self, host_tensor: torch.Tensor, device) -> None:
        """Keep a host tensor a kernel reads directly alive until the stream passes this point.
        A view into a sender's shared-memory segment is instead waited for here: the sender
        may rewrite the segment once the launching call has returned (shm_lease)."""
        ev = torch.cuda.Event()
        ev.record(current_stream(device))
        if shm_lease.aliases(host_tensor):
            ev.synchronize()
            return
        self._inflight.append((ev, host_tensor))


_staging = _Staging()

# Optional kernel timing hooks: when ``kernel_events`` is a list (bench.py), or while a
# flame_amd.metrics.KernelRecorder is active (``_recorders``), every native launch
# appends (name, start_event, end_event, algorithmic_bytes).  Events are recorded on
# the stream the kernel is launched on (torch's current stream).
kernel_events = None
_recorders = []


class _timed:
    def __init__(self, name, device, nbytes):
        self.name, self.device, self.nbytes = name, device, nbytes
        self.on = False

    def __enter__(self):
        self.on = kernel_events is not None or bool(_recorders)
        if self.on:
            self.e0 = torch.cuda.Event(enable_timing=True)
            self.e0.record(current_stream(self.device))
        return self

    def __exit__(self, *exc):
        if self.on and exc[0] is None:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record(current_stream(self.device))
            ev = (self.name, self.e0, e1, self.nbytes)
            if kernel_events is not None:
                kernel_events.append(ev)
            for r in _recorders:
                r.append(ev)
        return False


def _dev_index(device) -> int:
    device = torch.device(device) if not isinstance(device, torch.device) else device
    return device.index if device.index is not None else torch.cuda.current_device()


def _stream_ptr(device) -> int:
    """The raw HIP stream torch's current stream is on ``device`` (no Stream object made)."""
    return torch._C._cuda_getCurrentRawStream(_dev_index(device))


_STREAMS = {}


def current_stream(device) -> torch.cuda.Stream:
    """``torch.cuda.current_stream(device)``, the Stream object kept per (device, raw stream):
    torch's own call builds a new one each time, several per launch on the small-round path.
    (torch's pooled streams are never destroyed, so a raw pointer names one stream for good.)"""
    idx = _dev_index(device)
    key = (idx, torch._C._cuda_getCurrentRawStream(idx))
    st = _STREAMS.get(key)
    if st is None:
        st = _STREAMS[key] = torch.cuda.current_stream(idx)
    return st


def _keepalive(tensors, device):
    """Call AFTER the launch: device tensors join the stream's allocator bookkeeping,
    zero-copy host tensors are held until an event recorded behind the kernel fires."""
    st = current_stream(device)
    for t in tensors:
        if t.is_cuda:
            t.record_stream(st)
        else:
            _staging.hold(t, device)


def _device_ptrs(dev_meta: torch.Tensor, p: Plan):
    base = dev_meta.data_ptr()
    return base, base + p.off_clients, base + p.off_r32, base + p.off_r64


# ------------------------------------------------------------------ launches
# Zero-copy ingest: a pinned (hipHostMalloc'd) host tensor is device-addressable, so the
# kernel can stream client updates straight from host memory over PCIe instead of
# staging them into HBM first (FLAME_AMD_ZERO_COPY=0 disables).
ZERO_COPY_PINNED = os.environ.get("FLAME_AMD_ZERO_COPY", "1") != "0"


def _as_device(t: torch.Tensor, device) -> torch.Tensor:
    if t.device != device:
        if t.device.type == "cpu":
            shm_lease.check_live(t)     # a view of a sender's segment that has been rewritten raises
        if ZERO_COPY_PINNED and t.device.type == "cpu" and t.is_contiguous() and t.is_pinned():
            return t  # kept alive past the launch by _keepalive
        # a copy out of a sender's shared-memory segment completes before the call returns
        t = t.to(device, non_blocking=not shm_lease.aliases(t))
    return t.contiguous()


def tiled_stride(c: torch.Tensor, numel: int) -> int:
    """Bytes between chunks if ``c`` is a tiled slab view for a ``numel``-element
    aggregate (shape (ceil(numel/T), T), unit inner stride; see flame_amd/slab.py), else 0."""
    if c.dim() != 2 or not c.is_cuda or c.stride(1) != 1:
        return 0
    T = chunk_elems(dtype_code(c.dtype))
    if c.shape[1] != T or c.shape[0] != max(1, -(-numel // T)) or c.stride(0) < T:
        return 0
    return c.stride(0) * c.element_size()


def slice_elems(t: torch.Tensor, lo: int, hi: int, numel: int) -> torch.Tensor:
    """Elements [lo, hi) of a client tensor of ``numel`` logical elements, keeping a tiled
    slab view tiled (``lo`` must then be a multiple of the chunk)."""
    if t.is_cuda and tiled_stride(t, numel):
        T = t.shape[1]
        if lo % T:
            raise ValueError(f"tiled slice must start on a chunk boundary ({T})")
        return t[lo // T: -(-hi // T)]
    return t.reshape(-1)[lo:hi]


def _client_row(cs, o: torch.Tensor, device, keep):
    """Device pointers of one segment's clients + the segment's client_tile_stride.

    If every client is a tiled slab view with the same stride, the kernel reads
    them tiled; otherwise every client is read contiguous (tiled views that are
    mixed with other layouts in one call are copied out -- rare)."""
    n = o.numel()
    dt = o.dtype
    for c in cs:
        if c.dtype != dt:
            raise NotImplementedError(
                f"flame_amd: client tensor dtype {c.dtype} differs from aggregate dtype {dt}")
    if cs and cs[0].device == device:
        ts0 = tiled_stride(cs[0], n)
        if ts0:
            sh, st = cs[0].shape, cs[0].stride()
            if all(c.stride() == st and c.shape == sh and c.device == device for c in cs):
                if ts0 == chunk_elems(dtype_code(dt)) * o.element_size():
                    keep.extend(cs)   # ordinary contiguous (k, T) tensors: keep allocator bookkeeping
                # else: UpdateSlab views -- the slab outlives them, slot reuse is event-guarded
                return [c.data_ptr() for c in cs], ts0
    strides = [tiled_stride(c, n) if c.device == device else 0 for c in cs]
    row = []
    for c, ts in zip(cs, strides):
        if ts:
            c = c.reshape(-1)[:n]             # contiguous copy of a tiled view
        elif c.numel() != n:
            raise RuntimeError(f"flame_amd: client tensor has {c.numel()} elements, aggregate {n}")
        c = _as_device(c, device)
        keep.append(c)
        row.append(c.data_ptr() if c.is_cuda else host_device_pointer(c.data_ptr()))
    return row, 0


def host_device_pointer(host_ptr: int) -> int:
    """Device address of a pinned / hipHostRegister-ed host address (zero-copy reads)."""
    out = ctypes.c_void_p()
    N.check(N.lib().flame_host_device_pointer(host_ptr, ctypes.byref(out)))
    return int(out.value or 0)


def reduce_(outs: List[torch.Tensor], ins: Optional[List[torch.Tensor]], clients: List[List[torch.Tensor]],
            rates: Optional[Sequence[float]], *, init_first: bool = False,
            seg_rates: Optional[Sequence[Sequence[float]]] = None) -> None:
    """outs[s] = ins[s] (+)= Σ_i round(clients[s][i] * rates[i]) in order (kernel: flame_agg_reduce).

    ``outs`` are written in place (they must be contiguous device tensors);
    ``ins`` may be the same tensors (FedAvg mutates base_weights in place).
    ``seg_rates`` (instead of ``rates``) gives every segment its own rate row:
    independent reductions with equal client counts share one launch.
    """
    if not outs:
        return
    device = outs[0].device
    if device.type != "cuda":
        raise RuntimeError("flame_amd.reduce_: output tensors must live on the GPU (no CPU fallback)")
    groups = collections.OrderedDict()
    for s, o in enumerate(outs):
        groups.setdefault(dtype_code(o.dtype), []).append(s)
    keep = []
    for code, idx in groups.items():
        segs = []
        for s in idx:
            o = outs[s]
            assert o.is_contiguous() and o.device == device
            row, tstride = _client_row(clients[s], o, device, keep)
            inp = 0
            if not init_first:
                i_t = ins[s]
                assert i_t.is_contiguous() and i_t.device == device and i_t.numel() == o.numel()
                inp = i_t.data_ptr()
            segs.append(Seg(o.numel(), out=o.data_ptr(), inp=inp, clients=row, tile_stride=tstride))
        _launch_reduce(code, segs, rates if seg_rates is None else [seg_rates[s] for s in idx], device, keep,
                       init_first=init_first, seg_rates=seg_rates is not None)
    _keepalive(keep, device)


def _launch_reduce(code, segs, rates, device, keep, *, init_first=False, seg_rates=False) -> None:
    """One flame_agg_reduce launch over prepared segments (``keep`` holds what must outlive it)."""
    L = N.lib()
    flags = N.FLAME_AGG_INIT_FIRST if init_first else 0
    if seg_rates:
        flags |= N.FLAME_AGG_SEG_RATES
    n_cl = _n_clients(rates, seg_rates)
    nbytes = sum(s.numel for s in segs) * ITEMSIZE[code] * (n_cl + (1 if init_first else 2))
    est = compact_meta_bytes(code, len(segs), n_cl, seg_rates)
    if ARGMETA and est <= argmeta_max_bytes():
        # small launch: the metadata block goes with the dispatch as a kernel argument (no H2D blit)
        p = plan(code, segs, rates, seg_rates=seg_rates, compact=True)
        assert p.meta.nbytes == est
        with _timed("flame_agg_reduce", device, nbytes):
            N.check(L.flame_agg_reduce_argmeta(code, flags, p.meta.ctypes.data, p.meta.nbytes, p.n_segs,
                                               p.n_chunks, p.n_clients, p.off_clients, p.off_r32, p.off_r64,
                                               _stream_ptr(device)))
        return
    p = plan(code, segs, rates, seg_rates=seg_rates)
    if p.n_chunks >= XCD_MAP_MIN_CHUNKS and all(s.tile_stride == 0 for s in segs):
        # clients as separate tensors: each XCD streams a contiguous eighth of the chunks
        # (C3 rows 16.25 -> 15.89 ms; a tiled slab loses with it)
        flags |= N.FLAME_AGG_XCD_MAP
    dm = _staging.upload(p.meta, device)
    segp, clp, r32p, r64p = _device_ptrs(dm, p)
    with _timed("flame_agg_reduce", device, nbytes):
        N.check(L.flame_agg_reduce(code, flags, segp, p.n_segs, p.n_chunks, clp, p.n_clients, r32p, r64p,
                                   _stream_ptr(device)))
    keep.append(dm)


# Row-layout launches of at least this many chunks take the XCD-contiguous chunk map.
XCD_MAP_MIN_CHUNKS = int(os.environ.get("FLAME_AMD_XCD_MAP_MIN_CHUNKS", "4096"))

# Kernel-argument metadata for small launches (FLAME_AMD_ARGMETA=0 disables).
ARGMETA = os.environ.get("FLAME_AMD_ARGMETA", "1") != "0"
_ARGMETA_MAX = None


def argmeta_max_bytes() -> int:
    global _ARGMETA_MAX
    if _ARGMETA_MAX is None:
        _ARGMETA_MAX = int(N.lib().flame_agg_argmeta_max_bytes())
    return _ARGMETA_MAX


def compact_meta_bytes(code: int, n_segs: int, n_clients: int, seg_rates: bool = False) -> int:
    """Size of ``plan(..., compact=True)``'s block without building it: segments, client
    table and the one rate array the dtype reads (fp32 rates padded to 8 bytes)."""
    n_rates = (n_segs if seg_rates else 1) * n_clients
    return n_segs * (SEG_WORDS + n_clients) * 8 + (n_rates * 8 if code == N.FLAME_F64 else -(-n_rates // 2) * 8)


def _n_clients(rates, seg_rates) -> int:
    return len(rates[0]) if seg_rates else len(rates)


FEDOPT_VARIANT = {"fedadam": N.FLAME_FEDADAM, "fedyogi": N.FLAME_FEDYOGI, "fedadagrad": N.FLAME_FEDADAGRAD}


def fedopt_reduce_adapt_(variant: str, avg_out: List[Optional[torch.Tensor]], base: List[torch.Tensor],
                         cur: List[torch.Tensor], cur_out: List[torch.Tensor], m: List[torch.Tensor],
                         v: List[torch.Tensor], clients: List[List[torch.Tensor]], rates: Sequence[float],
                         hyper, state_zero: bool, cur_is_avg: Optional[Sequence[bool]] = None) -> None:
    """Fused FedAvg + FedOPT step (kernel: flame_fedopt_reduce_adapt), one launch per dtype
    (fp32 / bf16 / fp16; every tensor of a segment shares its dtype).  ``cur_is_avg[s]``:
    segment s's current weights ARE its FedAvg result (FLAME_SEG_CUR_IS_AVG: the caller's
    current aliases base, so d = avg - avg); ``cur[s]`` is then not read."""
    if not base:
        return
    device = base[0].device
    L = N.lib()
    groups = collections.OrderedDict()
    for s_, b in enumerate(base):
        groups.setdefault(dtype_code(b.dtype), []).append(s_)
    for code, idx in groups.items():
        segs, keep = [], []
        p_alias = 0
        for s_ in idx:
            alias = bool(cur_is_avg[s_]) if cur_is_avg is not None else False
            for t in (base[s_], cur_out[s_], m[s_], v[s_]) + (() if alias else (cur[s_],)):
                assert t.dtype == base[s_].dtype and t.is_contiguous() and t.device == device
            row, tstride = _client_row(clients[s_], base[s_], device, keep)
            segs.append(Seg(base[s_].numel(), out=avg_out[s_].data_ptr() if avg_out[s_] is not None else 0,
                            inp=base[s_].data_ptr(), cur=0 if alias else cur[s_].data_ptr(),
                            cur_out=cur_out[s_].data_ptr(), m=m[s_].data_ptr(), v=v[s_].data_ptr(), clients=row,
                            tile_stride=tstride, flags=N.FLAME_SEG_CUR_IS_AVG if alias else 0))
            p_alias += base[s_].numel() if alias else 0
        P = sum(sg.numel for sg in segs)
        isz = ITEMSIZE[code]
        # clients + base + cur (+ m, v unless zero state) read; avg, m, v, cur_out written
        nbytes = isz * (P * (len(rates) + 2 + (0 if state_zero else 2) + 4) - p_alias)
        h = list(hyper)
        if code in (N.FLAME_BF16, N.FLAME_F16):  # torch-CPU rounds the scalar of `sqrt(v) + tau`
            h[5] = float(torch.tensor(float(h[5]), dtype=base[idx[0]].dtype))
        opt_flags = N.FLAME_OPT_STATE_ZERO if state_zero else 0
        if ARGMETA and compact_meta_bytes(code, len(segs), len(rates)) <= argmeta_max_bytes():
            # small round: the metadata block rides in the kernel arguments (no H2D blit)
            p = plan(code, segs, rates, compact=True)
            with _timed("flame_fedopt_reduce_adapt", device, nbytes):
                N.check(L.flame_fedopt_reduce_adapt_argmeta(code, FEDOPT_VARIANT[variant], opt_flags,
                                                            p.meta.ctypes.data, p.meta.nbytes, p.n_segs,
                                                            p.n_chunks, p.n_clients, p.off_clients, p.off_r32,
                                                            *[float(x) for x in h], _stream_ptr(device)))
            _keepalive(keep, device)
            continue
        p = plan(code, segs, rates)
        dm = _staging.upload(p.meta, device)
        segp, clp, r32p, _ = _device_ptrs(dm, p)
        with _timed("flame_fedopt_reduce_adapt", device, nbytes):
            N.check(L.flame_fedopt_reduce_adapt(code, FEDOPT_VARIANT[variant], opt_flags,
                                                segp, p.n_segs, p.n_chunks, clp, p.n_clients, r32p,
                                                *[float(x) for x in h], _stream_ptr(device)))
        keep.append(dm)
        _keepalive(keep, device)


def fedopt_chain_(variant: str, base: List[torch.Tensor], cur: List[Optional[torch.Tensor]],
                  cur_out: List[torch.Tensor], m: List[torch.Tensor], v: List[torch.Tensor],
                  clients: List[List[torch.Tensor]], rates: Sequence[float], step_end: Sequence[bool], hyper,
                  state_zero: bool, first_aliased: Sequence[bool]) -> None:
    """A queue of eager FedOPT do() calls in one pass (kernel: flame_fedopt_chain), one launch
    per dtype (fp32 / bf16 / fp16; every tensor of a segment shares its dtype): per element,
    for each client in order, FedAvg into ``base`` (in place) with its rate, and after every
    client with ``step_end`` set, the adaptive step from the running current / m / v.
    ``first_aliased[s]``: segment s's current IS its base at the first step (``cur[s]`` unread);
    ``cur_out`` receives the final current, ``m`` / ``v`` are updated in place."""
    if not base:
        return
    device = base[0].device
    L = N.lib()
    if not step_end or not step_end[-1]:
        raise ValueError("fedopt_chain_: the last client must close a do() call")
    ends_host = np.asarray([1 if e else 0 for e in step_end], dtype=np.uint8)
    groups = collections.OrderedDict()
    for s_, b in enumerate(base):
        groups.setdefault(dtype_code(b.dtype), []).append(s_)
    for code, idx in groups.items():
        if code not in (N.FLAME_F32, N.FLAME_BF16, N.FLAME_F16):
            raise NotImplementedError(f"fedopt_chain_: dtype {base[idx[0]].dtype}")
    # every dtype group is planned and its tables uploaded BEFORE the first launch: a failure
    # there (a bad tensor, an allocation) leaves base / m / v untouched.  Only a
    # launch itself failing after another group's launch ran can leave the groups out of step;
    # that exception carries flame_partial = True (FedOPT then refuses further calls).
    launches = []
    for code, idx in groups.items():
        segs, keep = [], []
        p_alias = 0
        for s_ in idx:
            b = base[s_]
            alias = bool(first_aliased[s_])
            for t in (b, cur_out[s_], m[s_], v[s_]) + (() if alias else (cur[s_],)):
                assert t.dtype == b.dtype and t.is_contiguous() and t.device == device
            row, tstride = _client_row(clients[s_], b, device, keep)
            segs.append(Seg(b.numel(), out=b.data_ptr(), inp=b.data_ptr(), cur=0 if alias else cur[s_].data_ptr(),
                            cur_out=cur_out[s_].data_ptr(), m=m[s_].data_ptr(), v=v[s_].data_ptr(), clients=row,
                            tile_stride=tstride, flags=N.FLAME_SEG_CUR_IS_AVG if alias else 0))
            p_alias += b.numel() if alias else 0
        P = sum(sg.numel for sg in segs)
        # clients + base + cur (+ m, v unless zero state) read once; base, m, v, cur_out written once
        nbytes = ITEMSIZE[code] * (P * (len(rates) + 2 + (0 if state_zero else 2) + 4) - p_alias)
        h = list(hyper)
        if code in (N.FLAME_BF16, N.FLAME_F16):  # torch-CPU rounds the scalar of `sqrt(v) + tau`
            h[5] = float(torch.tensor(float(h[5]), dtype=base[idx[0]].dtype))
        p = plan(code, segs, rates)
        # the step_end bytes ride behind the plan's tables: one upload per launch
        pad = np.zeros(-(-ends_host.size // 8) * 8, dtype=np.uint8)
        pad[:ends_host.size] = ends_host
        dm = _staging.upload(np.concatenate([p.meta, pad.view(np.int64)]), device)
        keep.append(dm)
        launches.append((code, p, dm, h, nbytes, keep))
    for i, (code, p, dm, h, nbytes, keep) in enumerate(launches):
        segp, clp, r32p, _ = _device_ptrs(dm, p)
        try:
            with _timed("flame_fedopt_chain", device, nbytes):
                N.check(L.flame_fedopt_chain(code, FEDOPT_VARIANT[variant],
                                             N.FLAME_OPT_STATE_ZERO if state_zero else 0, segp, p.n_segs, p.n_chunks,
                                             clp, p.n_clients, r32p, dm.data_ptr() + p.meta.nbytes,
                                             *[float(x) for x in h], _stream_ptr(device)))
        except Exception as e:
            if i:
                e.flame_partial = True
            raise
        _keepalive(keep, device)


def fedopt_scalars(beta_1, beta_2, eta, tau):
    """fp32 scalars torch uses for `beta_1 * m`, `(1 - beta_1) * d`, ... (fedopt.py:113-129)."""
    f = np.float32
    return (f(beta_1), f(1 - beta_1), f(beta_2), f(1 - beta_2), f(eta), f(tau))


def scale_add_(bases: List[torch.Tensor], aggs: List[torch.Tensor], goal: int,
               deltas: Optional[List[torch.Tensor]] = None) -> None:
    """bases[s] += aggs[s] / goal in place; optional deltas[s] = new - old (flame_fedbuff_scale_add)."""
    if not bases:
        return
    device = bases[0].device
    L = N.lib()
    groups = collections.OrderedDict()
    for s, b in enumerate(bases):
        code = dtype_code(b.dtype) if b.is_floating_point() else None
        if code not in FLOAT_CODES:
            # torch: int_tensor / int -> float; in-place add into an int tensor raises
            raise RuntimeError(f"result type Float can't be cast to the desired output type "
                               f"{str(b.dtype).replace('torch.', '').capitalize()}")
        groups.setdefault(code, []).append(s)
    keep = []
    for code, idx in groups.items():
        segs = []
        for s in idx:
            b = bases[s]
            a = _as_device(aggs[s], device)
            if a.numel() != b.numel():
                raise RuntimeError(f"flame_amd: scale_add of {a.numel()} elements into {b.numel()}")
            if a.dtype != b.dtype:
                _scale_add_promoted(b, a, goal, deltas[s] if deltas is not None else None, device)
                continue
            keep.append(a)
            d = deltas[s].data_ptr() if deltas is not None else 0
            segs.append(Seg(b.numel(), out=b.data_ptr(), inp=a.data_ptr(), cur_out=d))
        if not segs:
            continue
        p = plan(code, segs, [], chunk=chunk_elems(code, scale_add=True))
        dm = _staging.upload(p.meta, device)
        nbytes = sum(s.numel for s in segs) * ITEMSIZE[code] * (3 + (1 if deltas is not None else 0))
        with _timed("flame_fedbuff_scale_add", device, nbytes):
            N.check(L.flame_fedbuff_scale_add(code, dm.data_ptr(), p.n_segs, p.n_chunks, int(goal),
                                              _stream_ptr(device)))
        keep.append(dm)
    _keepalive(keep, device)


def _scale_add_promoted(b: torch.Tensor, a: torch.Tensor, goal: int, delta, device) -> None:
    """``b += a / goal`` (fedbuff.py:126) when the aggregate's dtype is not the model's:
    ``q = a / goal`` is true division in a's dtype (int64 / int -> float32, torch's default
    dtype), formed by the scale_add kernel into a -0.0-filled buffer (x + -0 == x for every
    x, so the buffer holds exactly ``fl(a / goal)``); then the promoted in-place add
    (:func:`_add_promoted`); ``delta = new - old`` in b's dtype (common/util.py:152-159)."""
    af = a.reshape(-1)
    if not af.is_floating_point():
        af = af.to(torch.get_default_dtype())
    q = torch.full(af.shape, -0.0, dtype=af.dtype, device=device)
    scale_add_([q], [af], goal)
    old = b.clone() if delta is not None else None
    _add_promoted(b.view(-1), q)
    if delta is not None:
        from . import elementwise as ew
        dv = delta.view(-1)
        d = ew.Lazy.of(b.view(-1)) - ew.Lazy.of(old.view(-1))
        if d.dtype != dv.dtype:             # torch.sub(..., out=delta) casts into delta's dtype
            d = d.to(dv.dtype)
        if dv.is_cuda and dv.is_contiguous():
            ew.materialize(d, device=dv.device, into=[dv])
        else:
            dv.copy_(ew.materialize(d, device=device)[0])


# ------------------------------------------------------------------ co-located FedBuff hierarchy
HSEG_WORDS = N.HIER_SEGMENT_INT64S


@dataclass
class HierSeg:
    """One tensor of the hierarchy: the top's pointers + per-middle weight / delta pointers
    and the [n_mids * n_clients] arrival pointers (middle-major, arrival order)."""
    numel: int
    mid_w: Sequence[int]
    clients: Sequence[int]
    mid_delta: Optional[Sequence[int]] = None
    top_w: int = 0
    top_in: int = 0
    top_out: int = 0
    tile_stride: int = 0
    mid_tile_stride: int = 0   # bytes between chunks of one middle's weights (0 = contiguous)


@dataclass
class HierPlan:
    code: int
    meta: np.ndarray
    n_segs: int
    n_chunks: int
    n_mids: int
    n_clients: int
    offs: dict            # byte offsets of the tables inside the device copy of ``meta``


def _f32_words(x) -> np.ndarray:
    a = np.asarray(x, dtype=np.float64).reshape(-1).astype(np.float32)   # RNE, as torch rounds scalars
    if a.size % 2:
        a = np.concatenate([a, np.zeros(1, np.float32)])
    return a.view(np.int64)


def plan_hier(code: int, segs: Sequence[HierSeg], mid_rates, mid_goals, top_rates) -> HierPlan:
    """Device metadata of one flame_hier_fedbuff launch (no GPU needed):
    [segments (8 words)] [mid_w S x M] [mid_delta S x M] [clients S x M x C]
    [mid_rates f32 M x C] [mid_goal f32 M] [top_rates f32 M]."""
    S = len(segs)
    if S == 0:
        raise ValueError("empty segment list")
    M = len(mid_goals)
    if M == 0 or len(top_rates) != M or len(mid_rates) != M:
        raise ValueError("one goal, one top rate and one rate row per middle")
    C = len(mid_rates[0])
    if C == 0 or any(len(r) != C for r in mid_rates):
        raise ValueError("every middle needs the same (>= 1) number of arrivals")
    chunk = chunk_elems(code)
    head = np.zeros((S, HSEG_WORDS), dtype=np.uint64)
    wtab = np.empty((S, M), dtype=np.uint64)
    dtab = np.zeros((S, M), dtype=np.uint64)
    ctab = np.empty((S, M * C), dtype=np.uint64)
    begin = 0
    for i, s in enumerate(segs):
        if len(s.mid_w) != M or len(s.clients) != M * C or (s.mid_delta is not None and len(s.mid_delta) != M):
            raise ValueError("segment tables must be [n_mids] and [n_mids * n_clients]")
        wtab[i] = s.mid_w
        ctab[i] = s.clients
        if s.mid_delta is not None:
            dtab[i] = s.mid_delta
        fixed = [s.top_w, s.top_in, s.top_out]
        unaligned = (bool(np.any(ctab[i] % VEC_BYTES)) or bool(np.any(wtab[i] % VEC_BYTES))
                     or bool(np.any(dtab[i] % VEC_BYTES)) or any(p % VEC_BYTES for p in fixed if p))
        head[i] = (*fixed, s.numel, begin, N.FLAME_SEG_UNALIGNED if unaligned else 0, s.tile_stride,
                   s.mid_tile_stride)
        begin += -(-s.numel // chunk) if s.numel > 0 else 0
    if begin == 0:
        begin = 1
    parts = [head.view(np.int64).reshape(-1), wtab.view(np.int64).reshape(-1), dtab.view(np.int64).reshape(-1),
             ctab.view(np.int64).reshape(-1), _f32_words(mid_rates), _f32_words(mid_goals), _f32_words(top_rates)]
    names = ["segs", "mid_w", "mid_delta", "clients", "mid_rates", "mid_goal", "top_rates"]
    offs, o = {}, 0
    for nm, p in zip(names, parts):
        offs[nm] = o
        o += p.size * 8
    return HierPlan(code, np.concatenate(parts), S, begin, M, C, offs)


def hier_fedbuff_(segs: Sequence[HierSeg], code: int, mid_rates, mid_goals, top_rates, *, top_accum: bool,
                  top_goal: Optional[int], device, keep: list, mid_readonly: bool = False, sync: bool = False) -> None:
    """One flame_hier_fedbuff launch (the caller checked dtypes / devices / contiguity).
    ``sync``: the synchronous FedAvg hierarchy (FLAME_HIER_SYNC; needs ``top_accum``)."""
    L = N.lib()
    p = plan_hier(code, segs, mid_rates, mid_goals, top_rates)
    flags = ((N.FLAME_HIER_TOP_ACCUM if top_accum else 0) | (N.FLAME_HIER_TOP_APPLY if top_goal is not None else 0)
             | (N.FLAME_HIER_MID_READONLY if mid_readonly else 0) | (N.FLAME_HIER_SYNC if sync else 0))
    with_delta = any(s.mid_delta is not None for s in segs)
    P = sum(s.numel for s in segs)
    isz = ITEMSIZE[code]
    M, C = p.n_mids, p.n_clients
    # arrivals + middle weights (read, write) [+ deltas] + top (in) + top out [+ top weights r/w]
    # distinct middle-weight tensors (read-only middles may share one base: it is read once)
    wsum = sum(s.numel * len(set(int(p) for p in s.mid_w)) for s in segs)
    top_out = any(s.top_out for s in segs)
    nbytes = isz * (P * (M * C + (M if with_delta else 0) + (1 if top_accum else 0) + (1 if top_out else 0)
                         + (2 if top_goal is not None else 0)) + wsum * (1 if mid_readonly else 2))
    if ARGMETA and p.meta.nbytes <= argmeta_max_bytes():
        # small launch (e.g. one FedBuff aggregator's fused scale_add): metadata as a kernel argument
        o = p.offs
        with _timed("flame_hier_fedbuff", device, nbytes):
            N.check(L.flame_hier_fedbuff_argmeta(code, flags, p.meta.ctypes.data, p.meta.nbytes, p.n_segs, p.n_chunks,
                                                 M, C, o["mid_w"], o["mid_delta"] if with_delta else -1, o["clients"],
                                                 o["mid_rates"], o["mid_goal"], o["top_rates"], float(top_goal or 0),
                                                 _stream_ptr(device)))
        return
    dm = _staging.upload(p.meta, device)
    b = dm.data_ptr()
    with _timed("flame_hier_fedbuff", device, nbytes):
        N.check(L.flame_hier_fedbuff(code, flags, b + p.offs["segs"], p.n_segs, p.n_chunks, M, C,
                                     b + p.offs["mid_w"], b + p.offs["mid_delta"] if with_delta else None,
                                     b + p.offs["clients"], b + p.offs["mid_rates"], b + p.offs["mid_goal"],
                                     b + p.offs["top_rates"], float(top_goal or 0), _stream_ptr(device)))
    keep.append(dm)


def hier_resident_per_cu(code: int, n_mids: int, sync: bool = False) -> int:
    """Resident workgroups per CU of the flame_hier_fedbuff launch for these arguments."""
    r = int(N.lib().flame_hier_resident_per_cu(code, N.FLAME_HIER_SYNC if sync else 0, int(n_mids)))
    if r < 1:
        N.check(-r)
    return r


# ------------------------------------------------------------------ FedDyn server round
def feddyn_program(arrivals: Sequence, dict_order: Sequence, had_history) -> tuple:
    """Step program of one flame_feddyn_round launch (host only, no GPU).

    ``arrivals``: the ends in cache.iterkeys() order; ``dict_order``: local_param_dict's
    order after this round's untracked ends were appended (feddyn.py:125-139);
    ``had_history``: ends whose history existed (not None) before the round.  Returns
    ``([(flags, end), ...], n_phase1)``.  The FedAvg sum must run in arrival order and the
    history mean in dict order (feddyn.py:96-112).  When the arrivals appear in dict
    order in the same relative order, both sums ride one merged step list (each update
    and history read once); otherwise phase 1 walks the arrivals (average + history
    update) and phase 2 re-reads the histories in dict order for the mean."""
    arrived = set(arrivals)
    pos = {e: i for i, e in enumerate(dict_order)}
    ap = [pos[e] for e in arrivals]
    merged = all(a < b for a, b in zip(ap, ap[1:]))
    hist = [e for e in dict_order if e in arrived or e in had_history]

    def arrival(e):
        return N.FLAME_DYN_W | N.FLAME_DYN_AVG | N.FLAME_DYN_HOUT | (N.FLAME_DYN_HIN if e in had_history else 0)

    if merged:
        steps = [((arrival(e) | N.FLAME_DYN_MEAN) if e in arrived else (N.FLAME_DYN_HIN | N.FLAME_DYN_MEAN), e)
                 for e in hist]
        return steps, len(steps)
    steps = [(arrival(e), e) for e in arrivals] + [(N.FLAME_DYN_HIN | N.FLAME_DYN_MEAN, e) for e in hist]
    return steps, len(arrivals)


@dataclass
class DynSeg:
    """One tensor of a FedDyn round: base / average / cld pointers and, per program step,
    (w, h_in, h_out) pointers (0 where the step has none)."""
    numel: int
    out: int
    inp: int
    cld: int
    steps: Sequence[Sequence[int]]
    tile_stride: int = 0
    hist_tile_stride: int = 0


def plan_feddyn(code: int, segs: Sequence[DynSeg], flags: Sequence[int]):
    """[segments (8 words)] [steps S x K x 3] [flags u32 K] -> (meta, n_chunks, byte offsets)."""
    S, K = len(segs), len(flags)
    if S == 0 or K == 0:
        raise ValueError("feddyn plan needs >= 1 segment and >= 1 step")
    chunk = chunk_elems(code)
    head = np.zeros((S, N.DYN_SEGMENT_INT64S), dtype=np.uint64)
    tab = np.zeros((S, K * 3), dtype=np.uint64)
    begin = 0
    for i, s in enumerate(segs):
        if len(s.steps) != K:
            raise ValueError("every segment needs one pointer triple per step")
        tab[i] = np.asarray(s.steps, dtype=np.uint64).reshape(-1)
        unaligned = bool(np.any(tab[i] % VEC_BYTES)) or any(p % VEC_BYTES for p in (s.out, s.inp, s.cld))
        head[i] = (s.out, s.inp, s.cld, s.numel, begin, N.FLAME_SEG_UNALIGNED if unaligned else 0, s.tile_stride,
                   s.hist_tile_stride)
        begin += -(-s.numel // chunk) if s.numel > 0 else 0
    fl = np.asarray(flags, dtype=np.uint32)
    if fl.size % 2:
        fl = np.concatenate([fl, np.zeros(1, np.uint32)])
    parts = [head.view(np.int64).reshape(-1), tab.view(np.int64).reshape(-1), fl.view(np.int64)]
    offs = {"segs": 0, "steps": parts[0].size * 8, "flags": (parts[0].size + parts[1].size) * 8}
    return np.concatenate(parts), max(begin, 1), offs


def feddyn_round_(code: int, segs: Sequence[DynSeg], flags: Sequence[int], n_phase1: int, rate_avg: float,
                  rate_mean: float, device, keep: list) -> None:
    """One flame_feddyn_round launch (the caller checked dtypes / devices / contiguity)."""
    meta, n_chunks, offs = plan_feddyn(code, segs, flags)
    dm = _staging.upload(meta, device)
    b = dm.data_ptr()
    P = sum(s.numel for s in segs)
    reads = sum(bool(f & N.FLAME_DYN_W) + bool(f & N.FLAME_DYN_HIN) for f in flags)
    writes = sum(bool(f & N.FLAME_DYN_HOUT) for f in flags)
    nbytes = ITEMSIZE[code] * P * (reads + writes + 3)     # + base read, average and cld written
    with _timed("flame_feddyn_round", device, nbytes):
        N.check(N.lib().flame_feddyn_round(code, b + offs["segs"], len(segs), n_chunks, b + offs["steps"],
                                           b + offs["flags"], len(flags), n_phase1, float(rate_avg),
                                           float(rate_mean), _stream_ptr(device)))
    keep.append(dm)


def synth_fill_(out: torch.Tensor, seed: int, stream_id: int, start: int, sigma: float) -> None:
    """Fill a device tensor with flame_amd.synth values (bench / test inputs)."""
    from .synth import scale_for_sigma
    assert out.is_cuda and out.is_contiguous()
    N.check(N.lib().flame_synth_fill(dtype_code(out.dtype), out.data_ptr(), out.numel(), seed, stream_id,
                                     start, float(scale_for_sigma(sigma)), _stream_ptr(out.device)))


# ------------------------------------------------------------------ dict-level helpers used by the optimizers
def pick_device(*dicts) -> torch.device:
    for d in dicts:
        if d:
            for t in d.values():
                if isinstance(t, torch.Tensor) and t.is_cuda:
                    return t.device
    if not torch.cuda.is_available():
        raise RuntimeError("flame_amd: no HIP device available; the MI355X aggregation path has no CPU fallback")
    return torch.device("cuda", torch.cuda.current_device())


class _Target:
    """A tensor to be updated in place on the device; stages CPU / strided tensors."""

    def __init__(self, t: torch.Tensor, device):
        self.orig = t
        self.dev = t if (t.device == device and t.is_contiguous()) else t.to(device).contiguous()

    def writeback(self):
        if self.dev is not self.orig:
            self.orig.copy_(self.dev)


def accumulate(agg: dict, entries, *, device=None, key_groups=None, after_group=None) -> None:
    """agg[k] += round(v_i[k] * rate_i) for entries (weights, rate) in order, in place.

    Restates the per-client / per-key loop of fedavg.py:79-104 and fedbuff.py:89-97,
    136-157 (agg not None) as one launch per dtype over all keys and clients.

    ``key_groups`` (a partition of agg's keys, e.g. a parameter-sharded plan's waves):
    one launch per dtype per group, in group order, calling ``after_group(i)`` as soon
    as group ``i``'s launches are queued (the sharded path starts that group's
    all-gather there).  Pointer rows are still built once for all keys.
    """
    if not entries:
        return
    if device is None:   # the aggregate's own device first (no per-entry list for the common case)
        device = next((t.device for t in agg.values() if isinstance(t, torch.Tensor) and t.is_cuda), None) \
            or pick_device(*[w for w, _ in entries])
    if _accumulate_slab(agg, entries, device, key_groups, after_group):
        return
    if key_groups is not None:
        for w, _ in entries:
            for k in w.keys():
                if k not in agg:
                    raise KeyError(k)
        for gi, g in enumerate(key_groups):
            accumulate({k: agg[k] for k in g}, [({k: w[k] for k in g if k in w}, r) for w, r in entries],
                       device=device)
            if after_group is not None:
                after_group(gi)
        return
    keys = list(agg.keys())
    per_key = collections.OrderedDict()
    for ci, (w, _) in enumerate(entries):
        for k in w.keys():
            if k not in agg:
                raise KeyError(k)
            per_key.setdefault(k, []).append(ci)
    # group keys by participating-client set (normally every key has every client)
    groups = collections.OrderedDict()
    for k in keys:
        if k in per_key:
            groups.setdefault(tuple(per_key[k]), []).append(k)
    for cis, ks in groups.items():
        same = [k for k in ks if agg[k].dtype in DTYPE_CODE
                and all(entries[ci][0][k].dtype == agg[k].dtype for ci in cis)]
        mixed = [k for k in ks if k not in same]
        if same:
            targets = [_Target(agg[k], device) for k in same]
            outs = [t.dev for t in targets]
            clients = [[entries[ci][0][k] for ci in cis] for k in same]
            reduce_(outs, outs, clients, [entries[ci][1] for ci in cis])
            for t in targets:
                t.writeback()
        _accumulate_mixed(agg, mixed, [entries[ci] for ci in cis], device)


def weight_dtype(weights, k) -> torch.dtype:
    """dtype of ``weights[k]`` without making a view (slab slots know it from the slab)."""
    slab = getattr(weights, "slab", None)
    if slab is not None:
        rng = getattr(weights, "ranges", None)
        return slab.meta[rng[k][0] if rng is not None else k][0]
    return weights[k].dtype


def representatives(ws):
    """One weights dict per distinct layout among ``ws``: slots of one slab (sharing one
    ``ranges`` table) all carry the same keys and dtypes, so one of them stands for all;
    any other dict stands for itself.  Lets per-key dtype checks skip thousands of slots."""
    seen, out = set(), []
    for w in ws:
        slab = getattr(w, "slab", None)
        if slab is not None:
            tag = (id(slab), id(getattr(w, "ranges", None)), len(w))
            if tag in seen:
                continue
            seen.add(tag)
        out.append(w)
    return out


def slab_rows(ws, keys, numels, dtypes, device):
    """Pointer rows of ``keys`` for client weights ``ws`` that all live in ONE UpdateSlab:
    every ``w`` a whole :class:`~flame_amd.slab.SlotWeights` of the slab, or every ``w`` a
    :class:`~flame_amd.slab.SlabRef` sharing one ``ranges`` table.  Addresses come from the
    slot numbers (numpy), no per-client view is touched.  Returns ``{k: (uint64 pointers in
    ``ws`` order, tile stride bytes)}``, or None when the case does not apply (the caller
    then takes the per-view path)."""
    if not ws:
        return None
    first = ws[0]
    slab = getattr(first, "slab", None)
    if slab is None or slab.device != device:
        return None
    ranges = getattr(first, "ranges", None)
    nk = len(slab.keys)
    for w in ws:
        if getattr(w, "slab", None) is not slab or getattr(w, "ranges", None) is not ranges:
            return None
        if ranges is None and len(w) != nk:
            return None
    slots = np.fromiter((w.slot for w in ws), dtype=np.uint64, count=len(ws))
    return slot_rows(slab, ranges, slots, keys, numels, dtypes, device)


def slot_rows(slab, ranges, slots, keys, numels, dtypes, device):
    """:func:`slab_rows` from slot numbers already known (``slots``: uint64, client order) of
    ``slab`` (whole slots with ``ranges`` None, or one shared ``ranges`` table)."""
    if slab.device != device:
        return None
    rows = {}
    for k in keys:
        if ranges is not None:
            if k not in ranges:
                return None
            key, lo, hi = ranges[k]
        else:
            if k not in slab.meta:
                return None
            key, lo, hi = k, 0, slab.meta[k][2]
        dt, _, base, slot_bytes, tile_bytes = slab.key_layout(key)
        T = slab.storage[dt].shape[2]
        if dt != dtypes[k] or hi - lo != numels[k] or lo % T:
            return None
        rows[k] = (np.uint64(base + (lo // T) * tile_bytes) + slots * np.uint64(slot_bytes), tile_bytes)
    return rows


def _accumulate_slab(agg: dict, entries, device, key_groups=None, after_group=None) -> bool:
    """Fast path: every entry lives in ONE UpdateSlab (whole slots, or :class:`SlabRef`
    ranges sharing one table) and carries exactly agg's keys in agg's dtypes.  Pointer rows
    are computed from slot numbers (numpy), without touching the per-client views; returns
    False (nothing done) when the case does not apply."""
    w0 = entries[0][0]
    if getattr(w0, "slab", None) is None or len(w0) != len(agg):
        return False
    rows = slab_rows([w for w, _ in entries], list(agg.keys()), {k: agg[k].numel() for k in agg},
                     {k: agg[k].dtype for k in agg}, device)
    if rows is None:
        return False
    rates = [r for _, r in entries]
    targets = {k: _Target(agg[k], device) for k in agg.keys()}
    keep = []
    for gi, g in enumerate(key_groups if key_groups is not None else [list(agg.keys())]):
        groups = collections.OrderedDict()
        for k in g:
            groups.setdefault(dtype_code(agg[k].dtype), []).append(k)
        for code, ks in groups.items():
            segs = []
            for k in ks:
                ptrs, tile_bytes = rows[k]
                o = targets[k].dev
                segs.append(Seg(o.numel(), out=o.data_ptr(), inp=o.data_ptr(), clients=ptrs, tile_stride=tile_bytes))
            _launch_reduce(code, segs, rates, device, keep)
        if after_group is not None:
            after_group(gi)
    _keepalive(keep, device)
    for t in targets.values():
        t.writeback()
    return True


def _accumulate_mixed(agg: dict, keys, entries, device) -> None:
    """:func:`_accumulate_promoted` for many keys at once: each key's whole arrival loop
    (``tmp = (v * rate).to(v.dtype); agg[k] += tmp`` per entry, fedavg.py:93-104 /
    fedbuff.py:147-157) is ONE flame_elementwise program written in place into agg[k], and the
    keys whose dtypes / 0-dim-ness agree share one program and one launch (e.g. a ResNet's 53
    BatchNorm ``num_batches_tracked``: int64 updates into the fp32 aggregate FedOPT's promotion
    left).  Aggregates that are not contiguous device tensors, and entries holding tiled slab
    slots, take the per-key path."""
    from . import elementwise as ew
    rates = tuple(float(r) for _, r in entries)
    groups = collections.OrderedDict()
    for k in keys:
        acc = agg[k]
        vs = [w[k] for w, _ in entries]
        for v in vs:
            _check_cast(acc.dtype, v.dtype)
        if (not (acc.is_cuda and acc.device == device and acc.is_contiguous())
                or any(tuple(v.shape) != tuple(acc.shape) for v in vs) or len(vs) > ew.MAX_BUFS - 2):
            _accumulate_promoted(agg, k, entries, device)
            continue
        sig = (acc.dtype, acc.dim() == 0, tuple((v.dtype, v.dim() == 0) for v in vs), rates)
        groups.setdefault(sig, []).append(k)
    for sig, ks in groups.items():
        def stmt(acc, *vs):
            for v, r in zip(vs, rates):
                tmp = v * r
                acc = (acc + tmp.to(v.dtype)).to(acc.dtype)       # agg[k] += tmp, in place
            return acc
        k0 = ks[0]
        specs = [(agg[k0].dtype, tuple(agg[k0].shape))] + [(w[k0].dtype, tuple(w[k0].shape)) for w, _ in entries]
        try:
            prog = ew.cached(("accumulate",) + sig, stmt, specs)
        except NotImplementedError:      # a statement longer than one program: per key, as before
            for k in ks:
                _accumulate_promoted(agg, k, entries, device)
            continue
        prog.run_many([[agg[k]] + [w[k] for w, _ in entries] for k in ks], device, into=[[agg[k]] for k in ks])


def _accumulate_promoted(agg: dict, k, entries, device) -> None:
    """agg[k] += tmp_i where tmp_i = (v_i * rate_i).to(v_i.dtype) has another dtype than
    agg[k], or either is a dtype the kernels do not carry (:data:`NARROW`).

    Each tmp_i is formed in its own dtype (fedavg.py:93-102, :func:`tmp_of`), then added
    with torch's in-place semantics (:104): the sum in promote_types(acc, tmp), rounded back
    to acc's dtype -- :func:`_add_promoted` (integer aggregates: exact integer adds).  Runs
    of tmps whose promotion is acc's own float dtype (e.g. an fp32 aggregate receiving int64
    ``num_batches_tracked``) are summed in one launch: ``fl(acc + T(tmp))`` ==
    ``fl(acc + fl(T(tmp) * 1.0))``.
    """
    acc = agg[k]
    direct = acc.dtype in DTYPE_CODE
    terms = []                   # (tensor, rate, summable by the kernel into acc)
    for w, r in entries:
        v = w[k]
        _check_cast(acc.dtype, v.dtype)
        tmp = tmp_of(v, r, device, acc.shape)
        p = torch.promote_types(acc.dtype, tmp.dtype)
        if direct and p == acc.dtype and p.is_floating_point:    # integers: exact adds below
            terms.append((tmp if tmp.dtype == acc.dtype else tmp.to(acc.dtype), 1.0, True))
        else:
            terms.append((tmp, None, False))
    target = _Target(acc, device)
    run, run_r = [], []

    def flush_run():
        if run:
            reduce_([target.dev], [target.dev], [list(run)], list(run_r))
            run.clear()
            run_r.clear()
    for t, r, summable in terms:
        if summable:
            run.append(t)
            run_r.append(r)
        else:
            flush_run()
            _add_promoted(target.dev, t)
    flush_run()
    target.writeback()


def tmp_of(v: torch.Tensor, rate: float, device, shape=None) -> torch.Tensor:
    """``(v * rate).to(v.dtype)`` (fedavg.py:93-102) as a new device tensor.  Kernel dtypes:
    one init-first launch.  bool / uint8 / int8 / int16: ``v * rate`` is in torch's default
    dtype (fp32: the integral tensor and the rate both cast to it), formed by that dtype's kernel, then
    cast to v's dtype on the device (bool: != 0; integers: truncation -- in range, as
    ``|v * rate| <= |v|`` for the callers' rates <= 1).  ``shape``: the key's model shape
    (``v`` may be a tiled slab view)."""
    shape = v.shape if shape is None else shape
    if v.dtype in DTYPE_CODE:
        tmp = torch.empty(shape, dtype=v.dtype, device=device)
        reduce_([tmp], None, [[v]], [rate], init_first=True)
        return tmp
    if v.dtype not in NARROW:
        dtype_code(v.dtype)          # raises: unsupported (complex, fp8, ...)
    # torch computes an integral tensor times a Python float in the DEFAULT dtype (fp32 unless
    # torch.set_default_dtype changed it; fp64 then uses the rate unrounded)
    ft = torch.get_default_dtype()
    vf = v.to(device).to(ft)
    tf = torch.empty(shape, dtype=ft, device=device)
    reduce_([tf], None, [[vf]], [rate], init_first=True)
    return tf.to(v.dtype)


def _check_cast(acc_dt, v_dt) -> None:
    p = torch.promote_types(acc_dt, v_dt)
    if not torch.can_cast(p, acc_dt):
        raise RuntimeError(f"result type {str(p).replace('torch.', '').capitalize()} can't be cast to the "
                           f"desired output type {str(acc_dt).replace('torch.', '').capitalize()}")


def _add_promoted(acc: torch.Tensor, tmp: torch.Tensor) -> None:
    """``acc += tmp`` in place with torch's semantics when the dtypes differ: computed in
    promote_types(acc, tmp) and rounded back to acc's dtype (bf16 += f32, f16 += bf16,
    f32 += f64, ...; integer promotions such as int32 += int64 wrap like torch's) -- one
    flame_elementwise launch (casts, the add, the cast back)."""
    from . import elementwise as ew
    _check_cast(acc.dtype, tmp.dtype)
    ew.iadd(acc, ew.Lazy.of(tmp))


def logical_shape(weights, k):
    """Shape of ``weights[k]`` as the model sees it (slab slots hand out tiled views)."""
    shapes = getattr(weights, "shapes", None)
    if shapes is not None and k in shapes:
        return shapes[k]
    return weights[k].shape


def logical_tensor(weights, k) -> torch.Tensor:
    """``weights[k]`` in its logical shape (a tiled slab view is untiled into a copy)."""
    v = weights[k]
    shape = tuple(logical_shape(weights, k))
    if tuple(v.shape) == shape:
        return v
    n = 1
    for d in shape:
        n *= d
    return v.reshape(-1)[:n].reshape(shape)


def first_tmp(weights: dict, rate: float, *, device=None) -> dict:
    """{k: round(v[k] * rate)} as new device tensors (fedbuff.py:139-140,154-155)."""
    device = device or pick_device(weights)
    out = collections.OrderedDict()
    ks = list(weights.keys())
    kern = [k for k in ks if weight_dtype(weights, k) in DTYPE_CODE]
    for k in ks:
        if k in kern:
            out[k] = torch.empty(logical_shape(weights, k), dtype=weight_dtype(weights, k), device=device)
        else:
            out[k] = tmp_of(weights[k], rate, device, logical_shape(weights, k))
    if kern:
        reduce_([out[k] for k in kern], None, [[weights[k]] for k in kern], [rate], init_first=True)
    return out
