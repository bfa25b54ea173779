"""Python front of the CPU oracle (TEST INFRASTRUCTURE ONLY).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline
leg may import this module, and only as the checker.  The product path in
``flame_amd/`` never imports it and has no CPU fallback.

It restates the reference optimizers' ``do()`` control flow (which entries are
popped, in which order, which rate, which None results) in Python and runs the
per-element arithmetic in ``fedagg_oracle.c`` (built into ``liboracle.so``).
References (``/root/reference/lib/python/flame/``):
  * FedAvg.do            optimizer/fedavg.py:49-87, _aggregate_pytorch :89-104
  * FedOPT.do            optimizer/fedopt.py:58-92, _adapt_pytorch :102-129
  * FedBuff.do           optimizer/fedbuff.py:59-99, scale_add :101-127, _aggregate :136-157
  * FedDyn               optimizer/feddyn.py:51-62 (save_state), :64-115 (do), :125-139 (add_to_hist)
  * Scaffold             optimizer/scaffold.py:58-90 (save_state), :92-139 (do), :141-150
  * FedGFT               optimizer/fedgft.py:27-58 (FedAvg.do + update_bias), bias.py:74-106
Parity of this oracle is pinned by ``tests/test_oracle_golden.py`` against
vectors produced by the real reference (``tests/golden/make_golden.py``).
"""
from __future__ import annotations

import ctypes
import math
import os
import subprocess
from collections import OrderedDict

import numpy as np
import torch

try:
    from . import consult
except ImportError:  # loaded as a top-level module
    import consult

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2, torch.float64: 3,
      torch.int64: 4, torch.int32: 5}
VARIANT = {"fedadam": 0, "fedyogi": 1, "fedadagrad": 2}

_lib = None


def lib():
    """The C restatement, as a checker: every call counts as a consultation (consult.py)."""
    consult.note()
    return _load()


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            subprocess.check_call(["make", "-s", "-C", HERE])
        L = ctypes.CDLL(LIB_PATH)
        vp, i64, f32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_float
        L.flame_oracle_reduce.argtypes = [ctypes.c_int, vp, i64, vp, vp, vp, ctypes.c_int, ctypes.c_int]
        L.flame_oracle_scale_add.argtypes = [ctypes.c_int, vp, vp, i64, i64, vp]
        L.flame_oracle_fedopt_adapt.argtypes = [ctypes.c_int, vp, vp, vp, vp, vp, i64] + [f32] * 6
        L.flame_oracle_synth_f32.argtypes = [ctypes.c_uint64, ctypes.c_uint64, i64, i64, f32, vp]
        for f in ("flame_oracle_reduce", "flame_oracle_scale_add", "flame_oracle_fedopt_adapt",
                  "flame_oracle_synth_f32"):
            getattr(L, f).restype = None
        _lib = L
    return _lib


def _cpu(t):
    return t.detach().to("cpu").contiguous()


# --------------------------------------------------------------------------- kernels
def reduce_tensor(acc: torch.Tensor, clients, rates, init_first=False) -> None:
    """acc (CPU, contiguous) += Σ_i round(v_i * rate_i), sequential in list order (in place)."""
    assert acc.is_contiguous() and acc.device.type == "cpu"
    if any(c.dtype != acc.dtype for c in clients) or acc.dtype in NARROW:
        assert not init_first, "init_first needs the aggregate's own kernel dtype (use tmp_tensor)"
        # fedavg.py:93-104 with v.dtype != agg.dtype: tmp = (v*rate).to(v.dtype), then
        # `agg += tmp`: torch adds in promote_types(agg, tmp) and rounds back to agg's dtype
        # (legal in place when that promotion can be cast back: bf16 += f32 is, int += f32 is not)
        for c, r in zip(clients, rates):
            c = _cpu(c)
            if c.dtype == acc.dtype and acc.dtype not in NARROW:
                reduce_tensor(acc, [c], [r])
                continue
            p = torch.promote_types(acc.dtype, c.dtype)
            if not torch.can_cast(p, acc.dtype):
                raise RuntimeError("result type can't be cast to the desired output type")
            add_promoted(acc, tmp_tensor(c, r))
        return
    n = len(clients)
    cl = [_cpu(c) for c in clients]
    ptrs = (ctypes.c_void_p * max(n, 1))(*[c.data_ptr() for c in cl])
    r32 = np.asarray([np.float32(r) for r in rates] or [0], dtype=np.float32)
    r64 = np.asarray([float(r) for r in rates] or [0], dtype=np.float64)
    lib().flame_oracle_reduce(DT[acc.dtype], acc.data_ptr(), acc.numel(), ptrs,
                              r32.ctypes.data, r64.ctypes.data, n, int(bool(init_first)))


NARROW = (torch.bool, torch.uint8, torch.int8, torch.int16)


def tmp_tensor(v: torch.Tensor, rate) -> torch.Tensor:
    """``(v * rate).to(v.dtype)`` on the CPU (fedavg.py:93-102, fedbuff.py:143-153).  bool /
    uint8 / int8 / int16: ``v * rate`` is fp32 (both operands cast to fp32), then the cast
    back: bool = (x != 0), integers truncate."""
    v = _cpu(v)
    if v.dtype in NARROW:
        tf = torch.empty(v.shape, dtype=torch.float32)
        reduce_tensor(tf, [v.to(torch.float32)], [rate], init_first=True)
        return tf.to(v.dtype)
    tmp = torch.empty(v.shape, dtype=v.dtype)
    reduce_tensor(tmp, [v], [rate], init_first=True)
    return tmp


def add_promoted(acc: torch.Tensor, tmp: torch.Tensor) -> None:
    """acc += tmp (CPU, in place) for tmp of another dtype, as torch does it: the sum in
    promote_types(acc, tmp) -- one correctly rounded add, here the C restatement with rate
    1 -- then the cast back to acc's dtype; integer promotions are an exact integer add."""
    p = torch.promote_types(acc.dtype, tmp.dtype)
    if p.is_floating_point:
        accp = acc if p == acc.dtype else acc.to(p)
        reduce_tensor(accp, [tmp.to(p)], [1.0])
        if accp is not acc:
            acc.copy_(accp)
    else:
        acc.copy_(acc.to(p) + tmp.to(p))


def scale_add_tensor(base: torch.Tensor, agg: torch.Tensor, goal: int, want_delta=False):
    assert base.is_contiguous() and base.device.type == "cpu"
    if not base.is_floating_point():
        # torch: int_tensor / int -> float32; `base += float` on an int tensor raises
        raise RuntimeError("result type Float can't be cast to the desired output type "
                           + str(base.dtype).replace("torch.", "").capitalize())
    a = _cpu(agg)
    if a.dtype != base.dtype:
        # fedbuff.py:126 across dtypes: q = agg / goal in agg's dtype (int -> float32), then
        # `base += q` promoted; the scale_add restatement on a -0.0 buffer gives fl(agg / goal)
        af = a if a.is_floating_point() else a.to(torch.float32)
        q = torch.full(af.shape, -0.0, dtype=af.dtype)
        scale_add_tensor(q, af, goal)
        old = base.clone()
        add_promoted(base, q)
        return base - old if want_delta else None
    delta = torch.empty_like(base) if want_delta else None
    lib().flame_oracle_scale_add(DT[base.dtype], base.data_ptr(), a.data_ptr(), base.numel(), int(goal),
                                 delta.data_ptr() if delta is not None else None)
    return delta


def fedopt_scalars(beta_1, beta_2, eta, tau):
    f = np.float32
    return (f(beta_1), f(1 - beta_1), f(beta_2), f(1 - beta_2), f(eta), f(tau))


def adapt_tensor(sort, avg, cur, m, v, hyper):
    """Returns new cur; m and v (CPU fp32 contiguous) are updated in place."""
    for t in (avg, cur, m, v):
        if t.dtype != torch.float32:
            raise TypeError("adapt_tensor: fp32 only (non-fp32 keys use the torch op sequence)")
    out = torch.empty_like(cur)
    lib().flame_oracle_fedopt_adapt(VARIANT[sort], _cpu(avg).data_ptr(), _cpu(cur).data_ptr(),
                                    m.data_ptr(), v.data_ptr(), out.data_ptr(), cur.numel(),
                                    *[float(x) for x in hyper])
    return out


def synth_f32(seed, stream, start, n, scale) -> np.ndarray:
    out = np.empty(n, dtype=np.float32)
    _load().flame_oracle_synth_f32(seed, stream, start, n, float(scale), out.ctypes.data)
    return out


# --------------------------------------------------------------------------- do() restatements
class OracleFedAvg:
    """fedavg.py:49-104 control flow over a cache with iterkeys()/pop()/__len__."""

    def __init__(self):
        self.agg_weights = None

    def do(self, base_weights, cache, *, total=0, version=0, **kwargs):
        assert base_weights is not None
        self.agg_weights = base_weights
        if len(cache) == 0 or total == 0:
            return None
        for k in list(cache.iterkeys()):
            tres = cache.pop(k)
            rate = tres.count / total
            for key, v in tres.weights.items():
                acc = self.agg_weights[key]
                reduce_tensor(acc, [v], [rate])
        return self.agg_weights


class OracleFedGFT(OracleFedAvg):
    """fedgft.py:27-58: FedAvg.do unchanged; update_bias restates bias.py:74-106 (server side)."""

    def __init__(self, fair, gamma, reg="l2"):
        super().__init__()
        self.fair = fair
        self.a = self.b = self.c = self.d = self.val = self.sign = 0.0

    def update_bias(self, dataset_sizes, local_biases):
        n = sum(dataset_sizes.values())
        wm = {t: sum([getattr(local_biases[e], t) * dataset_sizes[e] / n for e in local_biases])
              for t in ("a", "b", "c", "d", "val")}
        self.a, self.b, self.c, self.d = wm["a"], wm["b"], wm["c"], wm["d"]
        if self.fair in ("SP", "EOP"):
            self.val = wm["val"]
        self.sign = 0.0 if self.val == 0 else (1.0 if self.val > 0 else -1.0)

    def bias_terms(self):
        return [self.a, self.b, self.c, self.d, self.val, self.sign]

    def get_bias(self):
        return self.val


class OracleFedOPT(OracleFedAvg):
    """fedopt.py:58-129 with the three _delta_v variants."""

    def __init__(self, sort, beta_1=0.9, beta_2=0.99, eta=1e-2, tau=1e-3, sqrt_rn=False):
        super().__init__()
        self.sort = sort
        # sqrt_rn: the reference's statements with every fp32 / fp64 op correctly rounded, as the
        # C oracle and the kernels compute them -- an fp32 root via fp64, an all-fp64 key in numpy
        # (IEEE ops); torch-CPU's own fp32 sqrt is not correctly rounded (~0.6 % of values one ulp
        # off) and its fp64 step differs from IEEE on some CPUs (one element in 513 on the MI355X
        # box's EPYC, profiles/r06z_ew_debug.log)
        self.sqrt_rn = sqrt_rn
        self.beta_1, self.beta_2, self.eta, self.tau = beta_1, beta_2, eta, tau
        self.hyper = fedopt_scalars(beta_1, beta_2, eta, tau)
        self.current_weights = None
        self.m_t = None
        self.v_t = None

    def do(self, base_weights, cache, *, total=0, version=0, **kwargs):
        self.agg_weights = super().do(base_weights, cache, total=total, version=version)
        if self.agg_weights is None:
            return self.current_weights
        if self.current_weights is None:
            self.current_weights = self.agg_weights
            return self.current_weights
        avg, cur = self.agg_weights, self.current_weights
        first = self.m_t is None
        if first:
            self.m_t, self.v_t = {}, {}
        new = OrderedDict()
        for k in cur.keys():
            # the C kernel takes all-fp32 state; anything else (e.g. FedAdaGrad's v of an int64
            # buffer stays int64: `v + d**2` on int64) keeps the reference's torch op sequence
            if (avg[k].dtype == torch.float32 and cur[k].dtype == torch.float32
                    and (first or (self.m_t[k].dtype == torch.float32 and self.v_t[k].dtype == torch.float32))):
                if first:
                    self.m_t[k] = torch.zeros_like(avg[k])
                    self.v_t[k] = torch.zeros_like(avg[k])
                new[k] = adapt_tensor(self.sort, avg[k], cur[k], self.m_t[k], self.v_t[k], self.hyper)
            else:
                new[k] = self._adapt_torch(k, avg[k], cur[k], first)
        self.current_weights = new
        return self.current_weights

    def _adapt_torch(self, k, avg, cur, first):
        """Non-fp32 keys: the reference's own torch op sequence (fedopt.py:106-129 and the
        _delta_v variants), which carries its dtype promotions (int64 -> fp32, bf16 rounding)."""
        consult.note()
        b1, b2, eta, tau = self.beta_1, self.beta_2, self.eta, self.tau
        if self.sqrt_rn and avg.dtype == cur.dtype == torch.float64 and (
                first or (self.m_t[k].dtype == self.v_t[k].dtype == torch.float64)):
            return self._adapt_numpy64(k, avg, cur, first)
        d = avg - cur
        m = torch.zeros_like(d) if first else self.m_t[k]
        m = b1 * m + (1 - b1) * d
        v = torch.zeros_like(d) if first else self.v_t[k]
        if self.sort == "fedadam":
            v = b2 * v + (1 - b2) * d**2
        elif self.sort == "fedyogi":
            v = v - (1 - b2) * d**2 * torch.sign(v - d**2)
        else:
            v = v + d**2
        self.m_t[k], self.v_t[k] = m, v
        sq = torch.sqrt(v)
        if self.sqrt_rn and sq.dtype == torch.float32:
            sq = torch.sqrt(v.to(torch.float32).double()).float()
        return cur + eta * m / (sq + tau)


    def _adapt_numpy64(self, k, avg, cur, first):
        """_adapt_torch's statements for an all-fp64 key in numpy: IEEE double ops, the root
        correctly rounded, torch.sign as (0 < x) - (x < 0) (NaN and -0 give +0)."""
        with np.errstate(all="ignore"):     # overflows / NaNs are part of the sequence (IEEE)
            return self._numpy64_step(k, avg, cur, first)

    def _numpy64_step(self, k, avg, cur, first):
        b1, b2, eta, tau = self.beta_1, self.beta_2, self.eta, self.tau
        a, c = avg.numpy(), cur.numpy()
        d = a - c
        m = np.zeros_like(d) if first else self.m_t[k].numpy()
        m = b1 * m + (1 - b1) * d
        v = np.zeros_like(d) if first else self.v_t[k].numpy()
        if self.sort == "fedadam":
            v = b2 * v + (1 - b2) * (d * d)
        elif self.sort == "fedyogi":
            x = v - d * d
            v = v - (1 - b2) * (d * d) * ((0 < x).astype(np.float64) - (x < 0).astype(np.float64))   # torch.sign
        else:
            v = v + d * d
        self.m_t[k], self.v_t[k] = torch.from_numpy(np.array(m)), torch.from_numpy(np.array(v))
        return torch.from_numpy(np.array(c + eta * m / (np.sqrt(v) + tau)))


class OracleFedBuff:
    """fedbuff.py:59-157."""

    def __init__(self):
        self.agg_goal_weights = None

    def do(self, agg_goal_weights, cache, *, total=0, version=0, **kwargs):
        self.agg_goal_weights = agg_goal_weights
        none_start = agg_goal_weights is None
        if len(cache) == 0 or total == 0:
            return None
        for k in list(cache.iterkeys()):
            tres = cache.pop(k)
            rate = 1 / math.sqrt(1 + version - tres.version)
            if none_start:
                self.agg_goal_weights = {}
            for key, v in tres.weights.items():
                if none_start:
                    self.agg_goal_weights[key] = tmp_tensor(v, rate)
                else:
                    reduce_tensor(self.agg_goal_weights[key], [v], [rate])
        return self.agg_goal_weights

    def scale_add_agg_weights(self, base_weights, agg_goal_weights, agg_goal):
        for k in base_weights.keys():
            scale_add_tensor(base_weights[k], agg_goal_weights[k], agg_goal)
        return base_weights


def _same_float(acc, *others):
    return acc.is_floating_point() and all(o.dtype == acc.dtype for o in others)


class OracleFedDyn(OracleFedAvg):
    """feddyn.py:31-139.  Same-dtype float keys run through the C kernel
    (``h + w`` == ``h + round(w*1.0)``; ``0.0 + Σ rate*h`` == a zero start);
    keys whose dtypes differ or are integer keep the reference's torch ops."""

    def __init__(self, alpha=0.01):
        super().__init__()
        self.alpha = alpha
        self.local_param_dict = {}
        self.cld_model = None

    def save_state(self, state, **kwargs):
        if getattr(state, "value", state) == "pre":
            self.local_param_dict = {e: self.local_param_dict.get(e) for e in kwargs["active_ends"]}

    def do(self, base_weights, cache, *, total=0, version=0, **kwargs):
        assert base_weights is not None
        self.agg_weights = base_weights
        if len(cache) == 0 or total == 0:
            return None
        rate = 1 / len(cache)
        for k in list(cache.iterkeys()):
            tres = cache.pop(k)
            self._add_to_hist(k, tres.weights)
            for key, v in tres.weights.items():
                reduce_tensor(self.agg_weights[key], [v], [rate])
        avg = self.agg_weights
        rate = 1 / len(self.local_param_dict)
        hist = [h for h in self.local_param_dict.values() if h is not None]
        self.cld_model = {}
        for k in avg:
            if _same_float(avg[k], *[h[k] for h in hist]):
                mean = torch.zeros_like(avg[k])
                reduce_tensor(mean, [h[k] for h in hist], [rate] * len(hist))
                out = avg[k].clone()
                reduce_tensor(out, [mean], [1.0])
            else:
                mean = 0.0
                for h in hist:
                    mean = mean + rate * h[k]
                out = avg[k] + mean
            self.cld_model[k] = out
        return avg

    def _add_to_hist(self, end, w):
        h = self.local_param_dict.get(end)
        if h is None:
            self.local_param_dict[end] = {k: _cpu(v).clone() for k, v in w.items()}
            return
        for k in list(h.keys()):
            if _same_float(h[k], w[k]):
                reduce_tensor(h[k], [w[k]], [1.0])
            else:
                h[k] = h[k] + _cpu(w[k])


class OracleScaffold(OracleFedAvg):
    """scaffold.py:36-150: control variates folded into c_glob with rate 1/len(weight_dict),
    then FedAvg with rate 1/len(cache)."""

    def __init__(self, k=3):
        super().__init__()
        self.c_glob = None
        self.weight_dict = None

    def save_state(self, state, **kwargs):
        if getattr(state, "value", state) != "pre":
            return
        if "dataset_sizes" in kwargs:
            ds = kwargs["dataset_sizes"]
            tot, n = sum(ds.values()), len(ds)
            self.weight_dict = {e: (ds[e] / tot) * n for e in ds}
        if "glob_weights" in kwargs and self.c_glob is None:
            g = kwargs["glob_weights"]
            self.c_glob = {k: torch.zeros(g[k].shape, dtype=g[k].dtype) for k in g}

    def do(self, base_weights, cache, *, total=0, version=0, **kwargs):
        assert base_weights is not None
        if len(cache) == 0 or total == 0:
            return None
        control_cache = kwargs["control_cache"]
        if len(control_cache) != len(cache):
            return None
        rate = 1 / len(self.weight_dict)
        for k in list(control_cache.iterkeys()):
            for key, v in control_cache.pop(k).weights.items():
                c = self.c_glob[key]
                if v.dtype == c.dtype:
                    reduce_tensor(c, [v], [rate])
                else:
                    tmp = _cpu(v) * rate
                    c += tmp.to(dtype=c.dtype)
        self.agg_weights = base_weights
        rate = 1 / len(cache)
        for k in list(cache.iterkeys()):
            for key, v in cache.pop(k).weights.items():
                reduce_tensor(self.agg_weights[key], [v], [rate])
        return self.agg_weights


class ListCache:
    """Minimal diskcache.Cache stand-in (sorted iterkeys, pop) for oracle tests."""

    def __init__(self):
        self._d = {}

    def __setitem__(self, k, v):
        self._d[k] = v

    def __len__(self):
        return len(self._d)

    def iterkeys(self):
        return iter(sorted(self._d))

    def pop(self, k, default=None):
        return self._d.pop(k, default)
