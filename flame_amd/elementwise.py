"""The reference's torch statements for the keys the fused kernels do not take -- int buffers
(``num_batches_tracked``), mixed-dtype keys, fp64 / int8 / uint8 / int16 tensors -- run as
``flame_elementwise`` programs (include/flame_amd.h) instead of PyTorch ops.

A :class:`Lazy` tensor records the statement it is built by (``a - c``, ``beta * m + x``,
``torch.sqrt(v) + tau``, ``torch.sign(...)``, ``torch.zeros_like(d)``, ``.to(dtype)``); the
optimizers run their own reference-shaped code on Lazy operands (FedOPT's ``_delta_v_tensor``
of each variant included), and :func:`materialize` compiles the recorded DAG into one typed
program and launches it.  Every result dtype is taken from torch itself: each op is replayed on
``meta`` tensors of the operands' real shapes, so the promotion (int64 * float -> fp32, bf16 +
fp16 -> fp32, a 0-dim operand's lower priority, ...) and the errors (bool subtraction) are
torch's own.  The kernel then computes what torch-CPU computes for that dtype: operands cast to
the op's result dtype first, fp32 / fp64 ops rounded once, bf16 / fp16 ops in fp32 rounded once
to the dtype (a Python scalar used in fp32 by ``*`` and rounded to the dtype before ``+``),
integer ops wrapped to their width.

Reference statements (paths relative to /root/reference/lib/python/flame/):
  optimizer/fedopt.py:102-129 (+ fedadam.py:33-35, fedyogi.py:34-36, fedadagrad.py:33-35),
  optimizer/scaffold.py:141-150, optimizer/feddyn.py:90-113,125-139.
There is no PyTorch fallback: a statement the kernel cannot express (a broadcast, a division by
a scalar, a power other than 2) raises ``NotImplementedError``.
"""
from __future__ import annotations

import ctypes

import torch

from . import _native as N

# element type codes flame_elementwise takes (include/flame_amd.h)
EW_DTYPES = {torch.float32: N.FLAME_F32, torch.bfloat16: N.FLAME_BF16, torch.float16: N.FLAME_F16,
             torch.float64: N.FLAME_F64, torch.int64: N.FLAME_I64, torch.int32: N.FLAME_I32,
             torch.uint8: N.FLAME_U8, torch.int8: N.FLAME_I8, torch.int16: N.FLAME_I16, torch.bool: N.FLAME_BOOL}
(LOAD, STORE, ZERO, CAST, ADD, SUB, MUL, DIV, ADD_S, MUL_S, SQUARE, SIGN, SQRT) = range(13)
MAX_OPS, MAX_REGS, MAX_BUFS = 64, 32, 16


class EwOp(ctypes.Structure):
    """flame_ew_op."""
    _fields_ = [("op", ctypes.c_int32), ("dtype", ctypes.c_int32), ("dst", ctypes.c_int32), ("a", ctypes.c_int32),
                ("b", ctypes.c_int32), ("pad", ctypes.c_int32), ("scalar", ctypes.c_double)]


def _meta(x):
    return torch.empty(x.shape, dtype=x.dtype, device="meta") if isinstance(x, Lazy) else x


_REPLAYED = {}


def _replay(fn, *xs, kind=None):
    """fn on meta stand-ins of the Lazy operands: torch's own result dtype and shape (and errors).
    With ``kind``, the result dtype is cached per (kind, operand dtypes, which operands are 0-dim,
    Python scalar types, torch's default dtype) -- everything torch's promotion looks at -- and the
    shape is the operands' broadcast (a meta op costs ~0.1 ms; a FedOPT statement makes ~20)."""
    if kind is None:
        r = fn(*[_meta(x) for x in xs])
        return r.dtype, tuple(r.shape)
    sig = (kind, torch.get_default_dtype()) + tuple(
        (x.dtype, len(x.shape) == 0) if isinstance(x, Lazy) else type(x) for x in xs)
    dt = _REPLAYED.get(sig)
    if dt is None:
        dt = _REPLAYED[sig] = fn(*[_meta(x) for x in xs]).dtype
    shape = torch.broadcast_shapes(*[x.shape for x in xs if isinstance(x, Lazy)])
    return dt, tuple(shape)


def _scalar(x):
    return isinstance(x, (int, float)) and not isinstance(x, bool)


class Lazy:
    """One tensor-valued node of a recorded statement (a leaf tensor or an op on nodes)."""

    __slots__ = ("dtype", "shape", "kind", "args", "scalar", "tensor")

    def __init__(self, dtype, shape, kind, args=(), scalar=0.0, tensor=None):
        if dtype not in EW_DTYPES:
            raise NotImplementedError(f"flame_amd elementwise: dtype {dtype} is not supported")
        self.dtype, self.shape, self.kind, self.args = dtype, tuple(shape), kind, tuple(args)
        self.scalar, self.tensor = float(scalar), tensor

    @staticmethod
    def of(t: torch.Tensor) -> "Lazy":
        return Lazy(t.dtype, t.shape, "leaf", tensor=t)

    # ---------------------------------------------------------------- recording
    def _same_shape(self, shape, what):
        if tuple(shape) != self.shape:
            raise NotImplementedError(f"flame_amd elementwise: {what} broadcasts {self.shape} to {tuple(shape)}")

    def to(self, dtype):
        if dtype == self.dtype:
            return self
        return Lazy(dtype, self.shape, "cast", (self,))

    def _cast(self, dtype):
        return self.to(dtype)

    def _binary(self, other, kind, fn, rfn=None):
        if isinstance(other, Lazy):
            dt, shape = _replay(fn, self, other, kind=kind)
            self._same_shape(shape, kind)
            other._same_shape(shape, kind)
            return Lazy(dt, shape, kind, (self._cast(dt), other._cast(dt)))
        if isinstance(other, torch.Tensor):
            return self._binary(Lazy.of(other), kind, fn)
        if not _scalar(other):
            return NotImplemented
        dt, shape = _replay(rfn or fn, self, other, kind=(kind, rfn is not None))
        if kind == "add":
            return Lazy(dt, shape, "add_s", (self._cast(dt),), scalar=other)
        if kind == "sub":            # x - s == x + (-s) exactly (round-to-nearest is symmetric)
            return Lazy(dt, shape, "add_s", (self._cast(dt),), scalar=-other)
        if kind == "mul":
            return Lazy(dt, shape, "mul_s", (self._cast(dt),), scalar=other)
        raise NotImplementedError(f"flame_amd elementwise: {kind} by a scalar")

    def __add__(self, o):
        return self._binary(o, "add", lambda a, b: a + b)

    def __radd__(self, o):
        return self._binary(o, "add", lambda a, b: b + a, lambda a, b: b + a)

    def __sub__(self, o):
        return self._binary(o, "sub", lambda a, b: a - b)

    def __rsub__(self, o):       # s - x == (-x) + s exactly
        if isinstance(o, Lazy):
            return o - self
        return (-self)._binary(o, "add", lambda a, b: b - (-a), lambda a, b: b - (-a))

    def __mul__(self, o):
        return self._binary(o, "mul", lambda a, b: a * b)

    def __rmul__(self, o):
        return self._binary(o, "mul", lambda a, b: b * a, lambda a, b: b * a)

    def __truediv__(self, o):
        if not isinstance(o, (Lazy, torch.Tensor)):
            raise NotImplementedError("flame_amd elementwise: division by a scalar")
        return self._binary(o, "div", lambda a, b: a / b)

    def __neg__(self):
        dt, shape = _replay(lambda a: -a, self, kind="neg")
        return Lazy(dt, shape, "mul_s", (self._cast(dt),), scalar=-1.0)

    def __pow__(self, e):
        if e != 2:
            raise NotImplementedError(f"flame_amd elementwise: ** {e}")
        dt, shape = _replay(lambda a: a ** 2, self, kind="pow2")
        return Lazy(dt, shape, "square", (self._cast(dt),))

    @classmethod
    def __torch_function__(cls, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        if func is torch.zeros_like and not kwargs:
            x = args[0]
            return Lazy(x.dtype, x.shape, "zero")
        if func in (torch.sqrt, torch.Tensor.sqrt) and not kwargs:
            dt, shape = _replay(torch.sqrt, args[0], kind="sqrt")
            return Lazy(dt, shape, "sqrt", (args[0]._cast(dt),))
        if func in (torch.sign, torch.Tensor.sign) and not kwargs:
            dt, shape = _replay(torch.sign, args[0], kind="sign")
            return Lazy(dt, shape, "sign", (args[0]._cast(dt),))
        raise NotImplementedError(f"flame_amd elementwise: {getattr(func, '__name__', func)} is not supported")


_KIND_OP = {"add": ADD, "sub": SUB, "mul": MUL, "div": DIV, "add_s": ADD_S, "mul_s": MUL_S, "square": SQUARE,
            "sign": SIGN, "sqrt": SQRT}


def _compile(outs, targets, inputs=None):
    """(program, buffers) storing each Lazy of ``outs`` into the tensor at the same place of
    ``targets``: nodes in dependency order, a register per live value (freed after its last
    reader), a LOAD per leaf node.  ``inputs``: the leaf tensors in the buffer order to use
    (a traced Program's positional inputs); by default, order of first use."""
    order, seen = [], set()

    def visit(n):
        if id(n) in seen:
            return
        seen.add(id(n))
        for a in n.args:
            visit(a)
        order.append(n)
    for o in outs:
        visit(o)
    bufs, buf_of = [], {}
    for t in inputs or ():
        buf_of[id(t)] = len(bufs)
        bufs.append(t)
    for n in order:
        if n.kind == "leaf" and id(n.tensor) not in buf_of:
            if inputs is not None:
                raise ValueError("flame_amd elementwise: a leaf outside the traced inputs")
            buf_of[id(n.tensor)] = len(bufs)
            bufs.append(n.tensor)
    out_buf = list(range(len(bufs), len(bufs) + len(targets)))
    bufs += list(targets)
    if len(bufs) > MAX_BUFS:
        raise NotImplementedError(f"flame_amd elementwise: {len(bufs)} buffers in one statement (max {MAX_BUFS})")
    last = {}
    for i, n in enumerate(order):
        for a in n.args:
            last[id(a)] = i
    keep = {id(o) for o in outs}
    prog, reg, free = [], {}, list(range(MAX_REGS - 1, -1, -1))
    for i, n in enumerate(order):
        if not free:
            raise NotImplementedError(f"flame_amd elementwise: more than {MAX_REGS} live values")
        r = free.pop()
        dt = EW_DTYPES[n.dtype]
        if n.kind == "leaf":
            prog.append(EwOp(LOAD, dt, r, buf_of[id(n.tensor)], 0, 0, 0.0))
        elif n.kind == "zero":
            prog.append(EwOp(ZERO, dt, r, 0, 0, 0, 0.0))
        elif n.kind == "cast":
            prog.append(EwOp(CAST, dt, r, reg[id(n.args[0])], EW_DTYPES[n.args[0].dtype], 0, 0.0))
        else:
            b = reg[id(n.args[1])] if len(n.args) > 1 else 0
            prog.append(EwOp(_KIND_OP[n.kind], dt, r, reg[id(n.args[0])], b, 0, n.scalar))
        reg[id(n)] = r
        for a in {id(a): a for a in n.args}.values():      # operands this node read last
            if last[id(a)] == i and id(a) not in keep:
                free.append(reg[id(a)])
    for o, b in zip(outs, out_buf):
        prog.append(EwOp(STORE, EW_DTYPES[o.dtype], 0, b, reg[id(o)], 0, 0.0))
    if len(prog) > MAX_OPS:
        raise NotImplementedError(f"flame_amd elementwise: {len(prog)} ops in one statement (max {MAX_OPS})")
    return prog, bufs


def materialize(*outs, device=None, into=None):
    """Run the statements that built ``outs`` as ONE flame_elementwise launch on ``device`` (the
    first CUDA leaf's by default) and return their values as new device tensors -- or, with
    ``into`` (one tensor per output), store them in place there (torch's in-place ``x += ...``).
    Leaf tensors on another device are copied to it first."""
    from . import engine
    outs = [o if isinstance(o, Lazy) else Lazy.of(o) for o in outs]
    leaves = []

    def walk(n, seen):
        if id(n) in seen:
            return
        seen.add(id(n))
        if n.kind == "leaf":
            leaves.append(n)
        for a in n.args:
            walk(a, seen)
    seen = set()
    for o in outs:
        walk(o, seen)
    if device is None:
        device = next((lf.tensor.device for lf in leaves if lf.tensor.is_cuda), None)
        if device is None:
            device = engine.pick_device()
    numel = 1
    for s in outs[0].shape:
        numel *= s
    for n in list(leaves) + outs:
        k = 1
        for s in n.shape:
            k *= s
        if k != numel:
            raise NotImplementedError(f"flame_amd elementwise: shapes {n.shape} and {outs[0].shape} in one statement")
    for lf in leaves:               # contiguous device operands (plumbing copies, as torch's own ops make)
        t = lf.tensor
        if t.device != device:
            t = t.to(device)
        lf.tensor = t.contiguous()
    if into is not None:
        targets = list(into)
        for t, o in zip(targets, outs):
            if t.dtype != o.dtype or tuple(t.shape) != o.shape or t.device != device or not t.is_contiguous():
                raise NotImplementedError("flame_amd elementwise: in-place target of another dtype / shape / device")
    else:
        targets = [torch.empty(o.shape, dtype=o.dtype, device=device) for o in outs]
    prog, bufs = _compile(outs, targets)
    ops = (EwOp * len(prog))(*prog)
    ptrs = (ctypes.c_void_p * len(bufs))(*[b.data_ptr() for b in bufs])
    nbytes = sum(b.numel() * b.element_size() for b in bufs)
    with engine._timed("flame_elementwise", device, nbytes):
        N.check(N.lib().flame_elementwise(ops, len(prog), ptrs, len(bufs), numel, engine._stream_ptr(device)))
    engine._keepalive(bufs, device)
    return targets


def iadd(target: torch.Tensor, x: "Lazy") -> None:
    """torch's in-place ``target += x``: the sum in promote_types(target, x), cast back to
    target's dtype, written into ``target`` (directly when it is a contiguous device tensor,
    else through a device result copied in)."""
    expr = (Lazy.of(target) + x).to(target.dtype)
    if target.is_cuda and target.is_contiguous():
        materialize(expr, device=target.device, into=[target])
    else:
        target.copy_(materialize(expr)[0])


class _Slot:
    """A traced program's positional input (stands for the tensor passed at run time)."""

    def __init__(self, i):
        self.i = i


class Program:
    """A statement compiled once (:func:`trace`) and run on any tensors of the traced dtypes and
    0-dim-ness: the op list and the output dtypes are fixed; the launch only binds buffers.  All
    inputs of one run must have one shape (the outputs take it)."""

    def __init__(self, prog, n_in, out_dtypes):
        self.ops = (EwOp * len(prog))(*prog)
        self.n_ops, self.n_in, self.out_dtypes = len(prog), n_in, list(out_dtypes)

    def __reduce__(self):       # picklable (an optimizer that holds programs can be checkpointed)
        return (_program, ([(o.op, o.dtype, o.dst, o.a, o.b, o.pad, o.scalar) for o in self.ops], self.n_in,
                           self.out_dtypes))

    def __call__(self, *inputs, device):
        from . import engine
        if len(inputs) != self.n_in:
            raise TypeError(f"flame_amd elementwise: {len(inputs)} inputs for a program of {self.n_in}")
        shape = tuple(inputs[0].shape)
        ins = []
        for t in inputs:
            if tuple(t.shape) != shape:
                raise NotImplementedError(f"flame_amd elementwise: shapes {tuple(t.shape)} and {shape} in one statement")
            ins.append((t if t.device == device else t.to(device)).contiguous())
        outs = [torch.empty(shape, dtype=dt, device=device) for dt in self.out_dtypes]
        bufs = ins + outs
        ptrs = (ctypes.c_void_p * len(bufs))(*[b.data_ptr() for b in bufs])
        numel = ins[0].numel()
        with engine._timed("flame_elementwise", device, sum(b.numel() * b.element_size() for b in bufs)):
            N.check(N.lib().flame_elementwise(self.ops, self.n_ops, ptrs, len(bufs), numel,
                                              engine._stream_ptr(device)))
        engine._keepalive(bufs, device)
        return outs


    def run_many(self, rows, device, into=None):
        """The program over several input tuples (one per key) in ONE flame_elementwise_segments
        launch; returns one output tuple per row.  Each output dtype's results share one new
        device buffer (a row's outputs are views of it in the row's shape) -- or, with ``into``
        (per row, one contiguous device tensor per output, of its dtype and the row's shape), are
        written there (an output may be one of the row's inputs: element i is read before it is
        written)."""
        import numpy as np
        from . import engine
        if len(rows) == 1 and into is None:
            return [self(*rows[0], device=device)]
        ins = []
        for row in rows:
            if len(row) != self.n_in:
                raise TypeError(f"flame_amd elementwise: {len(row)} inputs for a program of {self.n_in}")
            shape = tuple(row[0].shape)
            if any(tuple(t.shape) != shape for t in row):
                raise NotImplementedError(f"flame_amd elementwise: shapes {[tuple(t.shape) for t in row]} in one statement")
            ins.append([(t if t.device == device else t.to(device)).contiguous() for t in row])
        numels = [row[0].numel() for row in ins]
        ends = np.cumsum(np.asarray(numels, dtype=np.int64))
        total = int(ends[-1])
        if into is None:
            flats = [torch.empty(total, dtype=dt, device=device) for dt in self.out_dtypes]
            outs, off = [], 0
            for row, n in zip(ins, numels):
                outs.append([f[off:off + n].view(row[0].shape) for f in flats])
                off += n
        else:
            flats, outs = [], [list(t) for t in into]
            for row, orow in zip(ins, outs):
                for o, dt in zip(orow, self.out_dtypes):
                    if (o.dtype != dt or tuple(o.shape) != tuple(row[0].shape) or o.device != device
                            or not o.is_contiguous()):
                        raise NotImplementedError("flame_amd elementwise: an output target of another dtype / shape")
        n_bufs = self.n_in + len(self.out_dtypes)
        table = np.asarray([[t.data_ptr() for t in row] + [o.data_ptr() for o in orow] for row, orow in zip(ins, outs)],
                           dtype=np.uint64).reshape(len(rows), n_bufs)
        meta = np.concatenate([table.view(np.int64).reshape(-1), ends])
        dm = engine._staging.upload(meta, device)
        base = dm.data_ptr()
        nbytes = sum(t.numel() * t.element_size() for row in ins + outs for t in row)
        with engine._timed("flame_elementwise_segments", device, nbytes):
            N.check(N.lib().flame_elementwise_segments(self.ops, self.n_ops, base, n_bufs, base + table.nbytes,
                                                       len(rows), total, engine._stream_ptr(device)))
        engine._keepalive([t for row in ins + outs for t in row] + [dm], device)
        return outs


def _program(ops, n_in, out_dtypes):
    return Program([EwOp(*o) for o in ops], n_in, out_dtypes)


def trace(fn, specs):
    """Record ``fn`` on one Lazy leaf per ``(dtype, shape)`` of ``specs`` and compile what it
    returns (a Lazy or a tuple of them) into a :class:`Program` taking those inputs in order."""
    slots = [_Slot(i) for i in range(len(specs))]
    leaves = [Lazy(dt, shape, "leaf", tensor=sl) for (dt, shape), sl in zip(specs, slots)]
    outs = fn(*leaves)
    outs = list(outs) if isinstance(outs, (tuple, list)) else [outs]
    targets = [_Slot(len(specs) + j) for j in range(len(outs))]
    prog, _ = _compile(outs, targets, inputs=slots)
    return Program(prog, len(specs), [o.dtype for o in outs])


_PROGRAMS = {}


def cached(key, fn, specs):
    """The Program traced from ``fn`` on ``specs``, kept per ``key`` (a process-wide cache; it is
    cleared when it reaches 512 entries)."""
    prog = _PROGRAMS.get(key)
    if prog is None:
        if len(_PROGRAMS) >= 512:
            _PROGRAMS.clear()
        prog = _PROGRAMS[key] = trace(fn, specs)
    return prog
