"""Child process of tests/test_pickle_vm.py::test_no_read_past_the_buffer_guard_page.

Places each payload so that its last byte is the last byte before a PROT_NONE page and
decodes it with the C loop: every truncation of a flame update payload, and random byte
mutations of short ones.  A read past the end faults (the parent sees a signal exit)."""
import ctypes
import mmap
import os
import sys

import cloudpickle
import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flame_amd import ingest  # noqa: E402

PAGE = mmap.PAGESIZE
libc = ctypes.CDLL(None, use_errno=True)
libc.mprotect.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
_keep = []


def guarded(data: bytes) -> memoryview:
    pages = (len(data) + PAGE - 1) // PAGE + 1
    m = mmap.mmap(-1, pages * PAGE)
    off = (pages - 1) * PAGE - len(data)
    m[off:off + len(data)] = data
    addr = ctypes.addressof(ctypes.c_char.from_buffer(m))
    if libc.mprotect(ctypes.c_void_p(addr + (pages - 1) * PAGE), PAGE, 0) != 0:
        raise OSError(ctypes.get_errno(), "mprotect")
    _keep.append(m)
    return memoryview(m)[off:off + len(data)]


def main():
    if "--lib" in sys.argv:          # another build of the C loop (e.g. the UBSan one)
        import importlib.util
        path = sys.argv[sys.argv.index("--lib") + 1]
        spec = importlib.util.spec_from_file_location("flame_amd._pickle_vm", path)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        ingest._VM = mod
    assert ingest._VM is not None
    g = torch.Generator().manual_seed(0)
    msgs = [{"weights": {"a": torch.randn(3, 4, generator=g), "b": torch.arange(5).to(torch.int16),
                         "c": torch.tensor(True)}, "n": 2000, "meta": ("x", 1.5, [None])},
            {"weights": {"w": torch.randn(20_000, generator=g)}, "n": 7}]
    checked = 0
    for proto in (2, 3, 4, 5):
        for msg in msgs:
            pl = cloudpickle.dumps(msg, protocol=proto)
            ingest.decode(guarded(pl))                      # whole: decodes
            step = 1 if len(pl) < 4096 else 7
            for L in list(range(0, min(len(pl), 2048), 1)) + list(range(2048, len(pl), step)):
                try:
                    ingest.decode(guarded(pl[:L]))
                except Exception:  # noqa: BLE001 -- must raise, must not fault
                    pass
                checked += 1
                if len(_keep) > 256:                         # unmap old buffers as we go
                    del _keep[:128]
    rng = np.random.default_rng(1)
    base = cloudpickle.dumps(msgs[0], protocol=5)
    for _ in range(3000):
        m = bytearray(base)
        for _ in range(int(rng.integers(1, 4))):
            m[int(rng.integers(len(m)))] = int(rng.integers(256))
        cut = int(rng.integers(len(m) // 2, len(m) + 1))
        try:
            ingest.decode(guarded(bytes(m[:cut])))
        except Exception:  # noqa: BLE001
            pass
        checked += 1
        if len(_keep) > 256:
            del _keep[:128]
    print(f"guard ok: {checked} buffers")


if __name__ == "__main__":
    main()
