"""Test-only stand-in for the `diskcache` package (absent from this image).

The reference optimizers import ``from diskcache import Cache`` at module top
(lib/python/flame/optimizer/abstract.py:20, fedavg.py:19, fedbuff.py:21).
This shim is used ONLY by ``tests/golden/make_golden.py`` in the build
container to import the reference optimizer and record golden vectors.
It never travels to the GPU box as part of the product path.

Semantics restated from diskcache's documented API (unpinned upstream):
``__setitem__`` stores a pickled value, ``iterkeys()`` yields keys in
database sort order (ORDER BY key -> sorted order for str keys), ``pop``
removes and returns the unpickled value, ``reset`` is accepted and ignored.
"""
import pickle


class Cache:
    def __init__(self, *args, **kwargs):
        self._d = {}

    def __setitem__(self, key, value):
        self._d[key] = pickle.dumps(value)

    def __getitem__(self, key):
        return pickle.loads(self._d[key])

    def __len__(self):
        return len(self._d)

    def __contains__(self, key):
        return key in self._d

    def iterkeys(self, reverse=False):
        return iter(sorted(self._d, reverse=reverse))

    def pop(self, key, default=None):
        if key not in self._d:
            return default
        return pickle.loads(self._d.pop(key))

    def reset(self, *args, **kwargs):
        return None

    def clear(self):
        self._d.clear()
