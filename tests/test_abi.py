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


def test_elementwise_validates_programs_without_gpu():
    """flame_elementwise checks a program on the host before any launch: registers defined
    before they are read and of the dtype the reading op says, buffers present, known ops."""
    from flame_amd import _native
    from flame_amd import elementwise as E
    L = _native.lib()
    fake = ctypes.c_void_p(4096)    # never dereferenced: every call below fails (or is empty) on the host
    bufs = (ctypes.c_void_p * 2)(fake, fake)

    def run(ops, numel=8):
        arr = (E.EwOp * len(ops))(*ops)
        return L.flame_elementwise(arr, len(ops), bufs, 2, numel, None)
    f32, i64 = _native.FLAME_F32, _native.FLAME_I64
    assert run([E.EwOp(E.ADD, f32, 0, 1, 2, 0, 0.0)]) == _native.FLAME_EINVAL          # reads undefined registers
    assert run([E.EwOp(E.LOAD, i64, 0, 0, 0, 0, 0.0), E.EwOp(E.SQRT, f32, 1, 0, 0, 0, 0.0)]) == _native.FLAME_EINVAL
    assert b"dtype" in L.flame_last_error()                                             # an int64 register read as fp32
    assert run([E.EwOp(E.LOAD, i64, 0, 0, 0, 0, 0.0), E.EwOp(E.SQRT, i64, 1, 0, 0, 0, 0.0)]) == _native.FLAME_EINVAL
    assert b"sqrt" in L.flame_last_error()
    assert run([E.EwOp(E.LOAD, f32, 0, 5, 0, 0, 0.0)]) == _native.FLAME_EINVAL          # no buffer 5
    assert run([E.EwOp(E.LOAD, f32, 0, 0, 0, 0, 0.0), E.EwOp(E.STORE, i64, 0, 1, 0, 0, 0.0)]) == _native.FLAME_EINVAL
    assert run([E.EwOp(99, f32, 0, 0, 0, 0, 0.0)]) == _native.FLAME_EINVAL
    assert run([E.EwOp(E.LOAD, 12, 0, 0, 0, 0, 0.0)]) == _native.FLAME_EINVAL           # unknown dtype
    ok = [E.EwOp(E.LOAD, i64, 0, 0, 0, 0, 0.0), E.EwOp(E.CAST, f32, 1, 0, i64, 0, 0.0),
          E.EwOp(E.SQRT, f32, 2, 1, 0, 0, 0.0), E.EwOp(E.STORE, f32, 0, 1, 2, 0, 0.0)]
    assert run(ok, numel=0) == _native.FLAME_OK                                          # valid, nothing to launch
    assert L.flame_elementwise(None, 65, bufs, 2, 8, None) == _native.FLAME_EINVAL


def test_elementwise_programs_follow_torch_promotion():
    """The recorded FedOPT statements compile to programs whose every result dtype is torch's
    own (no GPU: compile only)."""
    import torch
    from flame_amd import elementwise as E
    for da, dc in [(torch.int64, torch.int64), (torch.int32, torch.float32), (torch.float64, torch.float64),
                   (torch.bfloat16, torch.float16), (torch.uint8, torch.int64), (torch.float16, torch.float16)]:
        for shape in [(5,), ()]:
            a, c = torch.ones(shape, dtype=da), torch.zeros(shape, dtype=dc)
            d = E.Lazy.of(a) - E.Lazy.of(c)
            m = 0.9 * torch.zeros_like(d) + (1 - 0.9) * d
            y = torch.zeros_like(d)
            y = y - (1 - 0.99) * d ** 2 * torch.sign(y - d ** 2)
            new = E.Lazy.of(c) + 1e-2 * m / (torch.sqrt(y) + 1e-3)
            d2 = a - c
            m2 = 0.9 * torch.zeros_like(d2) + (1 - 0.9) * d2
            y2 = torch.zeros_like(d2)
            y2 = y2 - (1 - 0.99) * d2 ** 2 * torch.sign(y2 - d2 ** 2)
            new2 = c + 1e-2 * m2 / (torch.sqrt(y2) + 1e-3)
            assert (m.dtype, y.dtype, new.dtype) == (m2.dtype, y2.dtype, new2.dtype), (da, dc)
            prog, bufs = E._compile([m, y, new], [torch.empty(o.shape, dtype=o.dtype) for o in (m, y, new)])
            assert len(prog) <= E.MAX_OPS and len(bufs) <= E.MAX_BUFS
            assert max(op.dst for op in prog) < E.MAX_REGS
    import pytest
    with pytest.raises(RuntimeError):           # torch refuses bool subtraction; so does the recording
        E.Lazy.of(torch.ones(3, dtype=torch.bool)) - E.Lazy.of(torch.ones(3, dtype=torch.bool))
    with pytest.raises(NotImplementedError):
        E.Lazy.of(torch.ones(3)) + E.Lazy.of(torch.ones(2, 3))


def test_traced_programs_pickle():
    """An optimizer holding compiled elementwise programs stays picklable (checkpoints)."""
    import pickle
    import torch
    from flame_amd import elementwise as E
    from flame_amd.optimizers import optimizer_provider
    opt = optimizer_provider.get("fedyogi")
    p = E.trace(opt._adapt_statement, [(torch.int64, ()), (torch.int64, ())])
    q = pickle.loads(pickle.dumps(p))
    assert (q.n_ops, q.n_in, q.out_dtypes) == (p.n_ops, p.n_in, p.out_dtypes)
    assert [(o.op, o.dtype, o.dst, o.a, o.b, o.scalar) for o in q.ops] == \
        [(o.op, o.dtype, o.dst, o.a, o.b, o.scalar) for o in p.ops]
