"""Read/write golden fixtures (.npz holding arrays + a JSON ``__meta__`` blob).

Tensors are stored as numpy arrays; bf16 is stored as its uint16 bit pattern
and tagged ``bf16`` in ``meta["dtypes"]`` so readers can rebuild torch tensors.
"""
from __future__ import annotations

import hashlib
import json

import numpy as np

try:  # torch is optional for pure-numpy readers
    import torch
except Exception:  # pragma: no cover
    torch = None

_TORCH_NAME = {
    "float32": "f32", "bfloat16": "bf16", "float16": "f16", "float64": "f64",
    "int64": "i64", "int32": "i32", "int16": "i16", "int8": "i8", "uint8": "u8", "bool": "b1",
}


def tensor_to_np(t):
    """torch tensor -> (numpy array, short dtype tag)."""
    t = t.detach().cpu().contiguous()
    tag = _TORCH_NAME[str(t.dtype).replace("torch.", "")]
    if tag == "bf16":
        return t.view(torch.int16).numpy().view(np.uint16).copy(), tag
    return t.numpy().copy(), tag


def np_to_tensor(a, tag):
    a = np.array(a, copy=True, order="C")          # keeps 0-d shapes (ascontiguousarray would not)
    if tag == "bf16":
        return torch.from_numpy(a.view(np.int16)).view(torch.bfloat16)
    return torch.from_numpy(a)


def digest(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


class FixtureWriter:
    def __init__(self):
        self.arrays = {}
        self.meta = {"dtypes": {}}

    def put(self, name, t):
        if torch is not None and isinstance(t, torch.Tensor):
            a, tag = tensor_to_np(t)
        else:
            a = np.asarray(t)
            tag = str(a.dtype)
        self.arrays[name] = a
        self.meta["dtypes"][name] = tag

    def put_weights(self, prefix, w):
        self.meta.setdefault("keys", {})[prefix] = list(w.keys())
        for k, v in w.items():
            self.put(f"{prefix}/{k}", v)

    def put_digest(self, prefix, w, head=16):
        self.meta.setdefault("digests", {})[prefix] = {}
        self.meta.setdefault("keys", {})[prefix] = list(w.keys())
        for k, v in w.items():
            a, tag = tensor_to_np(v)
            self.meta["digests"][prefix][k] = {"sha256": digest(a), "dtype": tag,
                                               "shape": list(a.shape)}
            self.put(f"{prefix}/{k}/head", a.reshape(-1)[:head].copy())

    def save(self, path):
        blob = np.frombuffer(json.dumps(self.meta, sort_keys=True).encode(), dtype=np.uint8)
        np.savez_compressed(path, __meta__=blob, **self.arrays)


LOADS = 0   # golden fixtures opened this process (tests/conftest.py's oracle-evidence check)


class Fixture:
    def __init__(self, path):
        global LOADS
        LOADS += 1
        z = np.load(path, allow_pickle=False)
        self.meta = json.loads(bytes(z["__meta__"]).decode())
        self.arrays = {k: z[k] for k in z.files if k != "__meta__"}

    def get(self, name):
        tag = self.meta["dtypes"][name]
        a = self.arrays[name]
        if torch is not None and tag in ("f32", "bf16", "f16", "f64", "i64", "i32", "i16", "i8", "u8", "b1"):
            return np_to_tensor(a, tag)
        return a

    def weights(self, prefix):
        return {k: self.get(f"{prefix}/{k}") for k in self.meta["keys"][prefix]}
