"""The C-ABI library loads without a GPU and exports every symbol include/flame_amd.h declares."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "flame_amd.h")


def header_functions():
    src = open(HDR).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(flame_[a-z0-9_]+)\s*\(", src)))


def test_header_matches_binding_list():
    from flame_amd import _native
    assert header_functions() == sorted(_native.EXPORTS)


def test_library_exports_every_symbol():
    from flame_amd import _native
    if not os.path.exists(_native.LIB_PATH):
        from flame_amd import build
        build.build()
    out = subprocess.check_output(["nm", "-D", "--defined-only", _native.LIB_PATH], text=True)
    syms = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    missing = [f for f in header_functions() if f not in syms]
    assert not missing, missing


def test_library_loads_and_reports_constants():
    from flame_amd import _native, engine
    L = _native.lib()
    assert L.flame_abi_version() == 1
    for code, isz in engine.ITEMSIZE.items():
        ce = L.flame_chunk_elems(code)
        assert ce == engine.chunk_elems(code) and (ce * isz) % (256 * 16) == 0
    for code in engine.FLOAT_CODES:
        assert L.flame_scale_add_chunk_elems(code) == engine.chunk_elems(code, scale_add=True)
    assert L.flame_chunk_elems(99) == 0


def test_argument_validation_without_gpu():
    """Invalid arguments are rejected on the host with a message, before any HIP call."""
    from flame_amd import _native
    L = _native.lib()
    assert L.flame_agg_reduce(0, 0, None, 0, 1, None, 0, None, None, None) == _native.FLAME_EINVAL
    assert b"segment" in L.flame_last_error()
    assert L.flame_fedbuff_scale_add(0, 8, 1, 1, 0, None) == _native.FLAME_EINVAL
    assert b"goal" in L.flame_last_error()
    with pytest.raises(_native.FlameError):
        _native.check(L.flame_synth_fill(0, None, 5, 0, 0, 0, 1.0, None))


@pytest.mark.parametrize("struct,words", [("flame_segment", "SEGMENT_INT64S"),
                                          ("flame_hier_segment", "HIER_SEGMENT_INT64S"),
                                          ("flame_dyn_segment", "DYN_SEGMENT_INT64S")])
def test_segment_struct_size(struct, words):
    src = open(HDR).read()
    body = re.search(r"typedef struct %s \{(.*?)\} %s;" % (struct, struct), src, re.S).group(1)
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    fields = [ln for ln in body.split(";") if ln.strip()]
    from flame_amd import _native
    assert len(fields) == getattr(_native, words)  # every field is 8 bytes


def test_fedopt_and_host_entry_points_validate_without_gpu():
    from flame_amd import _native
    L = _native.lib()
    args = [0, 0, 0, None, 0, 1, None, 0, None] + [0.0] * 6 + [None]
    assert L.flame_fedopt_reduce_adapt(*args) == _native.FLAME_EINVAL
    args[0] = 4  # int64 has no FedOPT kernel, but argument checks come first
    assert L.flame_fedopt_reduce_adapt(*args) == _native.FLAME_EINVAL
    assert L.flame_host_register(None, 0) == _native.FLAME_EINVAL
    assert L.flame_host_unregister(None) == _native.FLAME_EINVAL
    assert L.flame_host_device_pointer(None, None) == _native.FLAME_EINVAL


def test_agg_reduce_rejects_unknown_flags_without_gpu():
    from flame_amd import _native
    L = _native.lib()
    fake = ctypes.c_void_p(4096)   # never dereferenced: flags are checked on the host first
    assert L.flame_agg_reduce(0, 8, fake, 1, 1, None, 0, None, None, None) == _native.FLAME_EINVAL
    assert b"unknown flags" in L.flame_last_error()


def test_feddyn_round_validates_without_gpu():
    from flame_amd import _native
    L = _native.lib()
    fake = ctypes.c_void_p(4096)   # never dereferenced: argument checks run on the host first
    assert L.flame_feddyn_round(0, None, 0, 1, None, None, 0, 0, 0.5, 0.5, None) == _native.FLAME_EINVAL
    assert L.flame_feddyn_round(0, fake, 1, 1, fake, None, 2, 0, 0.5, 0.5, None) == _native.FLAME_EINVAL
    assert b"step flag" in L.flame_last_error()
    assert L.flame_feddyn_round(0, fake, 1, 1, fake, fake, 2, 3, 0.5, 0.5, None) == _native.FLAME_EINVAL
    assert b"n_phase1" in L.flame_last_error()


def test_agg_reduce_argmeta_validates_without_gpu():
    from flame_amd import _native
    L = _native.lib()
    cap = L.flame_agg_argmeta_max_bytes()
    assert cap == 3584
    blk = (ctypes.c_uint64 * 64)()
    assert L.flame_agg_reduce_argmeta(0, 0, None, 80, 1, 1, 0, 80, -1, -1, None) == _native.FLAME_EINVAL
    assert L.flame_agg_reduce_argmeta(0, 0, blk, cap + 8, 1, 1, 0, 80, -1, -1, None) == _native.FLAME_EINVAL
    assert L.flame_agg_reduce_argmeta(0, 0, blk, 512, 1, 1, 100, 80, 96, -1, None) == _native.FLAME_EINVAL
    assert b"outside" in L.flame_last_error()
    assert L.flame_agg_reduce_argmeta(0, 0, blk, 512, 1, 1, 4, 80, -1, -1, None) == _native.FLAME_EINVAL
    assert b"rate" in L.flame_last_error()
    assert L.flame_agg_reduce_argmeta(0, 8, blk, 512, 1, 1, 4, 80, 112, -1, None) == _native.FLAME_EINVAL


def test_hier_fedbuff_argmeta_validates_without_gpu():
    from flame_amd import _native
    L = _native.lib()
    blk = (ctypes.c_uint64 * 64)()
    # every call below is invalid, so nothing is ever launched (the pointers in blk are zeros)
    args = [0, 0, blk, 512, 1, 1, 1, 2, 64, -1, 504, 88, 96, 104, 0.0, None]   # client table runs past 512 B
    assert L.flame_hier_fedbuff_argmeta(*args) == _native.FLAME_EINVAL
    assert b"outside" in L.flame_last_error()
    bad = list(args)
    bad[3] = 4096
    assert L.flame_hier_fedbuff_argmeta(*bad) == _native.FLAME_EINVAL
    bad = list(args)
    bad[1] = 16
    assert L.flame_hier_fedbuff_argmeta(*bad) == _native.FLAME_EINVAL
    assert b"unknown flags" in L.flame_last_error()


def test_fedopt_argmeta_validates_without_gpu():
    from flame_amd import _native
    L = _native.lib()
    blk = (ctypes.c_uint64 * 64)()
    hyper = [0.9, 0.1, 0.99, 0.01, 0.01, 0.001]
    # every call below is invalid, so nothing is ever launched (the pointers in blk are zeros)
    assert L.flame_fedopt_reduce_adapt_argmeta(0, 0, 0, blk, 512, 1, 1, 2, 504, 96, *hyper, None) == _native.FLAME_EINVAL
    assert b"outside" in L.flame_last_error()
    assert L.flame_fedopt_reduce_adapt_argmeta(0, 0, 0, blk, 4096, 1, 1, 2, 80, 96, *hyper, None) == _native.FLAME_EINVAL
    assert L.flame_fedopt_reduce_adapt_argmeta(0, 0, 4, blk, 512, 1, 1, 2, 504, 96, *hyper, None) == _native.FLAME_EINVAL
    assert b"unknown flags" in L.flame_last_error()
    assert L.flame_fedopt_reduce_adapt_argmeta(0, 7, 0, blk, 512, 1, 1, 2, 504, 96, *hyper, None) == _native.FLAME_ENOTSUP
