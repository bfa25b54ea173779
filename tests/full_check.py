"""Full-size parity helpers: EVERY element of a full-size (BASELINE config) launch against the C
oracle, streamed through host memory.  Test infrastructure only (it calls oracle/).

The updates live in a tiled UpdateSlab on the device (``[tiles][capacity][T]``).  A chunk of
tiles is transposed ON THE GPU to client-major ``[n][chunk elements]`` (a device copy), copied
to pinned host memory, and the oracle (``flame_oracle_reduce`` & co, oracle/fedagg_oracle.c:91)
runs on it in ``WORKERS`` threads, each over a contiguous element range (ctypes releases the
GIL), so a 1024 x 25M fp32 check (102.4 GB) takes tens of seconds instead of hours.
"""
from __future__ import annotations

import concurrent.futures as cf

import numpy as np
import torch

WORKERS = 16
DT_CODE = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}
NP_VIEW = {torch.float32: np.float32, torch.bfloat16: np.uint16, torch.float16: np.uint16}


def _lib():
    from oracle import oracle as O
    return O.lib()


def _pool():
    global _POOL
    try:
        return _POOL
    except NameError:
        _POOL = cf.ThreadPoolExecutor(WORKERS)
        return _POOL


def columns(storage: torch.Tensor, n: int, numel: int, chunk_tiles: int = 512):
    """Yield ``(e0, e1, host)`` over the first ``n`` slots of a tiled slab tensor
    ``[tiles][capacity][T]``: ``host`` is a pinned ``[n][e1 - e0]`` tensor (client-major,
    elements e0..e1 of every client), reused between iterations."""
    tiles, _, T = storage.shape
    buf = None
    for t0 in range(0, tiles, chunk_tiles):
        t1 = min(tiles, t0 + chunk_tiles)
        e0, e1 = t0 * T, min(numel, t1 * T)
        if e1 <= e0:
            break
        dev = storage[t0:t1, :n, :].permute(1, 0, 2).reshape(n, (t1 - t0) * T)[:, :e1 - e0].contiguous()
        if buf is None or buf.numel() < dev.numel():
            buf = torch.empty(dev.numel(), dtype=storage.dtype, pin_memory=True)
        host = buf[:dev.numel()].view(n, e1 - e0)
        host.copy_(dev)
        del dev
        yield e0, e1, host


def reduce_chunk(host: torch.Tensor, acc: np.ndarray, rates, dtype, init_first=False) -> None:
    """acc[e] (+)= sum_i tmp(host[i][e], rates[i]) in client order, the oracle's op sequence,
    in WORKERS threads over element ranges.  ``acc``: numpy array (dtype's bit view)."""
    L = _lib()
    n, m = host.shape
    esz = host.element_size()
    r32 = np.asarray(rates, dtype=np.float64).astype(np.float32)
    r64 = np.asarray(rates, dtype=np.float64)
    base = np.uint64(host.data_ptr()) + np.arange(n, dtype=np.uint64) * np.uint64(m * esz)
    code = DT_CODE[dtype]
    step = -(-m // WORKERS)

    def work(lo):
        hi = min(m, lo + step)
        ptrs = base + np.uint64(lo * esz)
        L.flame_oracle_reduce(code, acc.ctypes.data + lo * esz, hi - lo, ptrs.ctypes.data, r32.ctypes.data,
                              r64.ctypes.data, n, 1 if init_first else 0)
    list(_pool().map(work, range(0, m, step)))


def bits(t: torch.Tensor) -> np.ndarray:
    """A CPU tensor's elements as numpy (bf16 / f16 as their uint16 bit patterns)."""
    t = t.detach().cpu().contiguous()
    if t.dtype in (torch.bfloat16, torch.float16):
        return t.view(torch.int16).numpy().view(np.uint16)
    return t.numpy()


def mismatches(a: np.ndarray, b: np.ndarray) -> int:
    """Elements whose bit patterns differ."""
    assert a.shape == b.shape and a.dtype == b.dtype
    return int(np.count_nonzero(np.asarray(a).view(np.uint8).reshape(a.size, -1) !=
                                np.asarray(b).view(np.uint8).reshape(b.size, -1), axis=1).astype(bool).sum())


def fedopt_adapt(variant: str, avg: np.ndarray, cur: np.ndarray, m: np.ndarray, v: np.ndarray, hyper) -> np.ndarray:
    """flame_oracle_fedopt_adapt (fedopt.py:102-129 op sequence, fp32) in WORKERS threads:
    updates m / v in place, returns the new current weights."""
    from oracle import oracle as O
    L = _lib()
    out = np.empty_like(cur)
    n = avg.size
    step = -(-n // WORKERS)
    var = O.VARIANT[variant]

    def work(lo):
        hi = min(n, lo + step)
        L.flame_oracle_fedopt_adapt(var, avg.ctypes.data + 4 * lo, cur.ctypes.data + 4 * lo, m.ctypes.data + 4 * lo,
                                    v.ctypes.data + 4 * lo, out.ctypes.data + 4 * lo, hi - lo, *hyper)
    list(_pool().map(work, range(0, n, step)))
    return out


def scale_add(base: np.ndarray, agg: np.ndarray, goal: int, dtype, want_delta=False):
    """flame_oracle_scale_add (fedbuff.py:122-127 + the middle's delta) in place on ``base``;
    returns the delta (or None)."""
    L = _lib()
    n = base.size
    delta = np.empty_like(base) if want_delta else None
    esz = base.itemsize
    step = -(-n // WORKERS)
    code = DT_CODE[dtype]

    def work(lo):
        hi = min(n, lo + step)
        L.flame_oracle_scale_add(code, base.ctypes.data + esz * lo, agg.ctypes.data + esz * lo, hi - lo, goal,
                                 (delta.ctypes.data + esz * lo) if want_delta else None)
    list(_pool().map(work, range(0, n, step)))
    return delta


def close_fedopt(got: np.ndarray, ref: np.ndarray, tol=1e-6):
    """The SURVEY §8(c) FedOPT contract on whole arrays: elementwise relative error <= tol where
    |ref| >= tol * max|ref|, and rel-L2 <= tol.  Returns (max elementwise rel err, rel-L2)."""
    g, r = got.astype(np.float64), ref.astype(np.float64)
    big = np.abs(r) >= tol * np.abs(r).max()
    el = float((np.abs(g - r)[big] / np.abs(r)[big]).max()) if big.any() else 0.0
    l2 = float(np.linalg.norm(g - r) / max(np.linalg.norm(r), 1e-300))
    return el, l2

