"""Kernel metrics for flame's MetricCollector (tracing / metrics).

The reference times whole tasklets (``monitor/runtime.py:23-41`` saves
``runtime.<alias>`` in seconds into ``Role.mc``, a ``MetricCollector``,
``monitor/metric_collector.py:117-121``).  The drop-in optimizers add what the
aggregation itself did on the GPU: set ``optimizer.metric_collector = self.mc``
in the role (or pass any object with ``save(mtype, alias, value)``) and every
``do()`` / ``scale_add_agg_weights()`` records its native launches with HIP
events on the launch stream.  Reading an event's time needs the kernel to have
finished, so the numbers of a call are saved at the first later call that finds
them complete (or at :func:`flush`), never by synchronising inside ``do()``:

  ``runtime.<alias>.<kernel>``   seconds of device time in that call
  ``hbm_GBps.<alias>.<kernel>``  algorithmic HBM bytes / device time
  ``launches.<alias>.<kernel>``  number of launches

``<alias>`` defaults to the optimizer's class name in lower case.
"""
from __future__ import annotations

import collections
import contextlib
from typing import Dict, Iterable, List

from . import engine


class KernelRecorder(list):
    """Collects (name, start_event, end_event, bytes) of the native launches issued while
    active (``with KernelRecorder() as rec: ...``).  Recorders nest."""

    def __enter__(self):
        engine._recorders.append(self)
        return self

    def __exit__(self, *exc):
        engine._recorders.remove(self)
        return False

    def ready(self) -> bool:
        return all(e1.query() for _, _, e1, _ in self)

    def summary(self) -> Dict[str, dict]:
        return summarize(self)


def summarize(events: Iterable) -> Dict[str, dict]:
    """Per kernel: launches, total device seconds, algorithmic bytes, GB/s (events must be done)."""
    acc = collections.OrderedDict()
    for name, e0, e1, nbytes in events:
        d = acc.setdefault(name, {"launches": 0, "seconds": 0.0, "bytes": 0})
        d["launches"] += 1
        d["seconds"] += e0.elapsed_time(e1) / 1e3
        d["bytes"] += nbytes
    for d in acc.values():
        d["GBps"] = d["bytes"] / d["seconds"] / 1e9 if d["seconds"] > 0 else 0.0
    return acc


_pending: List[tuple] = []   # (mc, alias, recorder) waiting for their kernels to finish


def _save(mc, alias, rec) -> None:
    for name, d in summarize(rec).items():
        mc.save("runtime", f"{alias}.{name}", d["seconds"])
        mc.save("hbm_GBps", f"{alias}.{name}", d["GBps"])
        mc.save("launches", f"{alias}.{name}", d["launches"])


def submit(mc, alias: str, rec: KernelRecorder) -> None:
    """Queue a finished call's recorder; saves every queued recorder whose kernels are done."""
    if rec:
        _pending.append((mc, alias, rec))
    still = []
    for item in _pending:
        if item[2].ready():
            _save(*item)
        else:
            still.append(item)
    _pending[:] = still


def flush() -> None:
    """Wait for every queued call's kernels and save their metrics."""
    while _pending:
        mc, alias, rec = _pending.pop(0)
        rec[-1][2].synchronize()
        _save(mc, alias, rec)


@contextlib.contextmanager
def recording(owner):
    """Report the launches made inside the block to ``owner.metric_collector`` -- for work an
    optimizer queued in ``do()`` and launches later (a deferred aggregate reduced when it is
    first read), under the owner's alias like its own calls."""
    mc = getattr(owner, "metric_collector", None)
    if mc is None or getattr(owner, "_flame_amd_recording", False):
        yield
        return
    owner._flame_amd_recording = True
    try:
        with KernelRecorder() as rec:
            yield
    finally:
        owner._flame_amd_recording = False
    submit(mc, getattr(owner, "metric_alias", None) or type(owner).__name__.lower(), rec)


def instrument(fn):
    """Wrap an optimizer method so its launches are reported to ``self.metric_collector``."""
    import functools

    @functools.wraps(fn)
    def wrapper(self, *args, **kwargs):
        mc = getattr(self, "metric_collector", None)
        if mc is None or getattr(self, "_flame_amd_recording", False):
            return fn(self, *args, **kwargs)
        self._flame_amd_recording = True
        try:
            with KernelRecorder() as rec:
                out = fn(self, *args, **kwargs)
        finally:
            self._flame_amd_recording = False
        submit(mc, getattr(self, "metric_alias", None) or type(self).__name__.lower(), rec)
        return out

    return wrapper
