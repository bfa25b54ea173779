"""Replay the golden fixtures through any optimizer implementation.

The same drivers run the CPU oracle (tests/test_oracle_golden.py) and the HIP
path (tests/test_gpu_parity.py), reproducing the caller conventions recorded
in tests/golden/make_golden.py.  Each driver returns a list of
``(label, got_dict, expected_dict)`` for the checker.
"""
from __future__ import annotations

import hashlib
import math
from copy import deepcopy

import numpy as np
import torch

from fixture_io import tensor_to_np


class TR:
    """Duck-typed TrainResult(weights, count, version) (optimizer/train_result.py:19-26)."""

    def __init__(self, weights=None, count=0, version=0):
        self.weights, self.count, self.version = weights, count, version


class SortedCache:
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


def to_dev(w, device):
    return {k: v.to(device, copy=True) for k, v in w.items()}


def to_cpu(w):
    return {k: v.detach().cpu().clone() for k, v in w.items()}


def assert_bitwise(label, got, exp):
    assert list(got.keys()) == list(exp.keys()), label
    for k in exp:
        g, e = got[k].detach().cpu(), exp[k]
        assert g.dtype == e.dtype, f"{label}/{k}: dtype {g.dtype} vs {e.dtype}"
        assert g.shape == e.shape, f"{label}/{k}: shape {g.shape} vs {e.shape}"
        ga, _ = tensor_to_np(g)
        ea, _ = tensor_to_np(e)
        ga, ea = ga.reshape(-1), ea.reshape(-1)
        if not np.array_equal(ga.view(np.uint8), ea.view(np.uint8)):
            bad = np.flatnonzero(ga.reshape(-1) != ea.reshape(-1))
            raise AssertionError(f"{label}/{k}: {bad.size} elements differ, first at {bad[:5]}: "
                                 f"{ga.reshape(-1)[bad[:5]]} vs {ea.reshape(-1)[bad[:5]]}")


def assert_close_fedopt(label, got, exp, rtol=1e-6, elementwise=True):
    """SURVEY §8(c) FedOPT contract: per round from identical state, elementwise rel err <= rtol
    where |ref| >= rtol*max|ref|, and rel-L2 <= rtol; across rounds (state already differs by
    torch-CPU's sqrt ulps) rel-L2 <= rtol only (elementwise=False)."""
    for k in exp:
        assert got[k].shape == exp[k].shape, f"{label}/{k}: shape {got[k].shape} vs {exp[k].shape}"
        if exp[k].numel() == 0:
            continue
        g = got[k].detach().cpu().double()
        e = exp[k].double()
        den = e.abs()
        if den.max() == 0:       # an all-zero reference (e.g. m_t after d = 0): exactly zero
            assert torch.equal(g, e), f"{label}/{k}: expected all zeros"
            continue
        mask = den >= rtol * den.max()
        rel = ((g - e).abs()[mask] / den[mask]).max().item() if mask.any() else 0.0
        l2 = ((g - e).norm() / e.norm().clamp_min(1e-300)).item()
        assert rel <= rtol or not elementwise, f"{label}/{k}: max elementwise rel err {rel:.3e}"
        assert l2 <= rtol, f"{label}/{k}: rel-L2 {l2:.3e}"


# ---------------------------------------------------------------- drivers
def run_fedavg(fx, make_opt, device):
    m = fx.meta
    base = to_dev(fx.weights("base"), device)
    cache = SortedCache()
    for i, (e, c) in enumerate(zip(m["end_ids"], m["counts"])):
        cache[e] = TR(to_dev(fx.weights(f"client{i}"), device), c)
    assert list(cache.iterkeys()) == m["order"]
    opt = make_opt("fedavg")
    out = opt.do(base, cache, total=m["total"], num_trainers=m["n"])
    assert out is base, "FedAvg must return (and mutate) the base_weights object (fedavg.py:74,87)"
    assert len(cache) == 0, "cache entries must be consumed (fedavg.py:82)"
    return [("out", out, fx.weights("out"))]


def run_fedavg_synth(fx, make_opt, device):
    from flame_amd import synth
    m = fx.meta

    def gen(stream, sigma):
        shapes = m["shapes"]
        total = sum(int(np.prod(s)) for _, s in shapes)
        flat = synth.synth_f32(m["seed"], stream, total, sigma)
        out, off = {}, 0
        for k, s in shapes:
            n = int(np.prod(s))
            out[k] = torch.from_numpy(flat[off:off + n].copy()).reshape(s).to(device)
            off += n
        return out

    base = gen(m["base_stream"], m["sigma_base"])
    cache = SortedCache()
    for e, s, c in zip(m["end_ids"], m["client_streams"], m["counts"]):
        cache[e] = TR(gen(s, m["sigma_delta"]), c)
    out = make_opt("fedavg").do(base, cache, total=m["total"], num_trainers=2)
    for k, d in m["digests"]["out"].items():
        a, _ = tensor_to_np(out[k].cpu())
        assert list(a.shape) == d["shape"]
        assert hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest() == d["sha256"], \
            f"mnist2/{k}: digest mismatch"
    return []


def run_fedavg_eager(fx, make_opt, device):
    m = fx.meta
    opt = make_opt("fedavg")
    cache = SortedCache()
    base = to_dev(fx.weights("base"), device)
    total = 0
    res = []
    for step, (e, c) in enumerate(zip(m["end_ids"], m["counts"])):
        total += c
        cache[e] = TR(to_dev(fx.weights(f"client{step}"), device), c)
        out = opt.do(base, cache, total=total, num_trainers=m["n"])
        assert out is base
        res.append((f"after{step}", deepcopy(to_cpu(out)), fx.weights(f"after{step}")))
    return res


def run_none(fx, make_opt, device):
    opt = make_opt("fedavg")
    base = {"w": torch.ones(3, device=device)}
    assert (opt.do(deepcopy(base), SortedCache(), total=5) is None) == fx.meta["empty_is_none"]
    c = SortedCache()
    c["x"] = TR({"w": torch.ones(3, device=device)}, 0)
    assert (opt.do(deepcopy(base), c, total=0) is None) == fx.meta["total0_is_none"]
    assert len(c) == fx.meta["total0_cache_len_after"]
    return []


def run_fedbuff_seq(fx, make_opt, device):
    m = fx.meta
    opt = make_opt("fedbuff")
    agg = None
    res = []
    for i in range(m["goal"]):
        cache = SortedCache()
        cache[f"t{i}"] = TR(to_dev(fx.weights(f"update{i}"), device), m["counts"][i],
                            m["round"] - m["stale"][i])
        agg = opt.do(agg, cache, total=m["counts"][i], version=m["round"])
        res.append((f"agg{i}", deepcopy(to_cpu(agg)), fx.weights(f"agg{i}")))
    weights = to_dev(fx.weights("weights0"), device)
    new = opt.scale_add_agg_weights(weights, agg, m["goal"])
    assert new is weights, "scale_add mutates and returns base_weights (fedbuff.py:122-127)"
    res.append(("out", new, fx.weights("out")))
    return res


def run_fedbuff_subsets(fx, make_opt, device):
    """Arrivals with key subsets, one per do(); twice: the aggregate read only at the end
    (every arrival still queued in a deferred aggregate), then read after every arrival."""
    m = fx.meta
    res = []
    for read_each in (False, True):
        opt = make_opt("fedbuff")
        agg = None
        for i in range(m["goal"]):
            cache = SortedCache()
            cache[f"t{i}"] = TR(to_dev(fx.weights(f"update{i}"), device), 1, m["round"] - m["stale"][i])
            agg = opt.do(agg, cache, total=1, version=m["round"])
            if read_each:
                to_cpu(agg)
        res.append((f"agg/read_each={read_each}", to_cpu(agg), fx.weights("agg")))
        weights = to_dev(fx.weights("weights0"), device)
        new = opt.scale_add_agg_weights(weights, agg, m["goal"])
        res.append((f"out/read_each={read_each}", new, fx.weights("out")))
    return res


def run_fedbuff_dtypes(fx, make_opt, device):
    """Every-dtype FedBuff sequence: the aggregate after each arrival, then scale_add of the
    float keys."""
    m = fx.meta
    opt = make_opt("fedbuff")
    agg = None
    res = []
    for i in range(m["goal"]):
        cache = SortedCache()
        cache[f"t{i}"] = TR(to_dev(fx.weights(f"update{i}"), device), 1, m["round"] - m["stale"][i])
        agg = opt.do(agg, cache, total=1, version=m["round"])
        res.append((f"agg{i}", to_cpu(agg), fx.weights(f"agg{i}")))
    weights = to_dev(fx.weights("weights0"), device)
    new = opt.scale_add_agg_weights(weights, agg, m["goal"])
    res.append(("out", new, fx.weights("out")))
    return res


def run_downcast(fx, make_opt, device):
    """Updates of another dtype than the aggregate (torch adds in the promoted dtype and rounds
    back): FedAvg; FedBuff read after every arrival and read once at the end (all queued),
    each followed by a scale_add into a model of other dtypes."""
    m = fx.meta
    base = to_dev(fx.weights("fedavg/base"), device)
    cache = SortedCache()
    for i, (e, c) in enumerate(zip(m["end_ids"], m["counts"])):
        cache[e] = TR(to_dev(fx.weights(f"fedavg/client{i}"), device), c)
    assert list(cache.iterkeys()) == m["order"]
    out = make_opt("fedavg").do(base, cache, total=m["total"], num_trainers=m["n"])
    res = [("fedavg", out, fx.weights("fedavg/out"))]
    for read_each in (True, False):
        opt = make_opt("fedbuff")
        agg = None
        for i in range(m["goal"]):
            c = SortedCache()
            c[f"t{i}"] = TR(to_dev(fx.weights(f"fedbuff/update{i}"), device), 1, m["round"] - m["stale"][i])
            agg = opt.do(agg, c, total=1, version=m["round"])
            if read_each:
                res.append((f"fedbuff/agg{i}", to_cpu(agg), fx.weights(f"fedbuff/agg{i}")))
        w = to_dev(fx.weights("fedbuff/weights0"), device)
        new = opt.scale_add_agg_weights(w, agg, m["goal"])
        res.append(("fedbuff/out" + ("" if read_each else " (deferred)"), new, fx.weights("fedbuff/out")))
    return res


def run_narrow(fx, make_opt, device):
    """bool / uint8 / int8 / int16 buffers next to float keys: the downcast driver's FedAvg and
    FedBuff passes; a scale_add into a bool model raises as in the reference."""
    res = run_downcast(fx, make_opt, device)
    opt = make_opt("fedbuff")
    m = fx.meta
    agg = None
    for i in range(m["goal"]):
        c = SortedCache()
        c[f"t{i}"] = TR(to_dev(fx.weights(f"fedbuff/update{i}"), device), 1, m["round"] - m["stale"][i])
        agg = opt.do(agg, c, total=1, version=m["round"])
    try:
        opt.scale_add_agg_weights({"mask": to_dev(fx.weights("fedavg/base"), device)["mask"]}, agg, m["goal"])
        raised = False
    except RuntimeError:
        raised = True
    assert raised == m["scale_add_bool_raises"]
    return res


def run_fedbuff_none_multi(fx, make_opt, device):
    m = fx.meta
    cache = SortedCache()
    for i, k in enumerate(["k0", "k1", "k2"]):
        cache[k] = TR(to_dev(fx.weights(f"update{i}"), device), 10, m["versions"][i])
    out = make_opt("fedbuff").do(None, cache, total=10, version=m["round"])
    return [("out", out, fx.weights("out"))]


def run_fedopt(fx, make_opt, device):
    m = fx.meta
    opt = make_opt(m["sort"], beta_1=m["beta_1"], beta_2=m["beta_2"], eta=m["eta"], tau=m["tau"])
    weights = to_dev(fx.weights("weights0"), device)
    res = []
    for r in range(m["rounds"]):
        cache = SortedCache()
        for i, c in enumerate(m["counts"][r]):
            cache[f"r{r}c{i}"] = TR(to_dev(fx.weights(f"r{r}/client{i}"), device), c)
        # reference caller: do(deepcopy(self.weights), ...) then self.weights = result
        weights = opt.do(deepcopy(weights), cache, total=sum(m["counts"][r]), num_trainers=m["n"])
        res.append((f"r{r}/cur", to_cpu(weights), fx.weights(f"r{r}/cur")))
        res.append((f"r{r}/avg", to_cpu(opt.agg_weights), fx.weights(f"r{r}/avg")))
        if f"r{r}/m" in fx.meta["keys"]:
            res.append((f"r{r}/m", to_cpu(opt.m_t), fx.weights(f"r{r}/m")))
            res.append((f"r{r}/v", to_cpu(opt.v_t), fx.weights(f"r{r}/v")))
    return res


def run_fedopt_eager(fx, make_opt, device):
    """The eager top aggregator's FedOPT calls (make_golden.fedopt_eager): per round one
    base = deepcopy(weights), then do(base, cache, total=running) per arrival."""
    m = fx.meta
    opt = make_opt(m["sort"], beta_1=m["beta_1"], beta_2=m["beta_2"], eta=m["eta"], tau=m["tau"])
    weights = to_dev(fx.weights("weights0"), device)
    res = []
    for r, rc in enumerate(m["counts"]):
        base = deepcopy(weights)
        cache = SortedCache()
        total = 0
        for i, c in enumerate(rc):
            total += c
            cache[f"r{r}e{i}"] = TR(to_dev(fx.weights(f"r{r}/client{i}"), device), c)
            out = opt.do(base, cache, total=total, num_trainers=len(rc))
            res.append((r, f"r{r}/a{i}/out", to_cpu(out), fx.weights(f"r{r}/a{i}/out")))
            res.append((r, f"r{r}/a{i}/base", to_cpu(base), fx.weights(f"r{r}/a{i}/base")))
            if f"r{r}/a{i}/m" in m["keys"]:
                res.append((r, f"r{r}/a{i}/m", to_cpu(opt.m_t), fx.weights(f"r{r}/a{i}/m")))
                res.append((r, f"r{r}/a{i}/v", to_cpu(opt.v_t), fx.weights(f"r{r}/a{i}/v")))
        weights = out
    return res


FEDOPT_EAGER_FIXTURES = ["fedadam_eager.npz", "fedyogi_eager.npz"]


def check_fedopt_eager(res):
    """Round 0 (passthrough, then d = 0 while current aliases base, then one adaptive step
    from identical state): the §8(c) single-round contract; round 1: rel-L2 (state drift)."""
    for r, label, got, exp in res:
        assert_close_fedopt(label, got, exp, elementwise=(r == 0))


def hier_shape(m):
    """(middles, arrivals per middle, the top's version of each middle) of a hier fixture."""
    mids, arr = m.get("mids", 2), m.get("arrivals", 3)
    return mids, arr, m.get("mid_versions", [m["round"] - i for i in range(mids)])


def run_hier(fx, make_opt, device, delta_fn):
    m = fx.meta
    rnd = m["round"]
    mids, arr, mver = hier_shape(m)
    top_w0 = fx.weights("top_w0")
    res = []
    deltas = []
    for mid in range(mids):
        opt = make_opt("fedbuff")
        mid_w = to_dev(top_w0, device)
        agg = None
        for t in range(arr):
            cache = SortedCache()
            cache[f"m{mid}t{t}"] = TR(to_dev(fx.weights(f"m{mid}/update{t}"), device), 10 + t, rnd - t % 2)
            agg = opt.do(agg, cache, total=10 + t, version=rnd)
        prev = deepcopy(mid_w)
        mid_w = opt.scale_add_agg_weights(mid_w, agg, arr)
        delta = delta_fn(mid_w, prev)
        res.append((f"m{mid}/delta", to_cpu(delta), fx.weights(f"m{mid}/delta")))
        deltas.append(delta)
    opt = make_opt("fedbuff")
    agg = None
    for mid, d in enumerate(deltas):
        cache = SortedCache()
        cache[f"mid{mid:02d}"] = TR(d, 30, mver[mid])
        agg = opt.do(agg, cache, total=30, version=rnd)
    top = opt.scale_add_agg_weights(to_dev(top_w0, device), agg, mids)
    res.append(("top_out", to_cpu(top), fx.weights("top_out")))
    return res


HIER_FIXTURES = ["hier_fedbuff_small.npz", "hier_fedbuff_wide.npz"]


def run_hier_fedavg(fx, make_opt, device):
    """Synchronous hierarchy as separate calls (make_golden.hier_fedavg_small): per middle
    FedAvg.do(deepcopy(w), cache, total) + delta; top FedAvg.do over the deltas."""
    m = fx.meta
    top = to_dev(fx.weights("top_w0"), device)
    mids = [to_dev(fx.weights("top_w0"), device) for _ in range(3)]
    res = []
    for r, rm in enumerate(m["rounds"]):
        top_cache = SortedCache()
        totals = []
        for j, mm in enumerate(rm["mids"]):
            cache = SortedCache()
            for i, (e, c) in enumerate(zip(mm["ids"], mm["counts"])):
                cache[e] = TR(to_dev(fx.weights(f"r{r}/m{j}/client{i}"), device), c)
            assert list(cache.iterkeys()) == mm["order"]
            new = make_opt("fedavg").do(deepcopy(mids[j]), cache, total=sum(mm["counts"]))
            delta = {k: new[k] - mids[j][k] for k in new}
            mids[j] = new
            res.append((f"r{r}/m{j}/new", to_cpu(new), fx.weights(f"r{r}/m{j}/new")))
            res.append((f"r{r}/m{j}/delta", to_cpu(delta), fx.weights(f"r{r}/m{j}/delta")))
            top_cache[f"mid{j}"] = TR(delta, sum(mm["counts"]))
            totals.append(sum(mm["counts"]))
        assert list(top_cache.iterkeys()) == rm["top_order"]
        top = make_opt("fedavg").do(deepcopy(top), top_cache, total=sum(totals))
        res.append((f"r{r}/top", to_cpu(top), fx.weights(f"r{r}/top")))
    return res


def run_hier_fedavg_fused(fx, device, with_delta=True, slab=False):
    """The same rounds through flame_amd.optimizer.sync_hierarchy.sync_hierarchy_round (GPU)."""
    from flame_amd.optimizer.sync_hierarchy import sync_hierarchy_round
    m = fx.meta
    top = to_dev(fx.weights("top_w0"), device)
    mids = [to_dev(fx.weights("top_w0"), device) for _ in range(3)]
    store = None
    if slab:
        from flame_amd.slab import UpdateSlab
        store = UpdateSlab(fx.weights("top_w0"), capacity=16, device=device)
    res = []
    for r, rm in enumerate(m["rounds"]):
        specs = []
        for j, mm in enumerate(rm["mids"]):
            cache = SortedCache()
            for i, (e, c) in enumerate(zip(mm["ids"], mm["counts"])):
                w = to_dev(fx.weights(f"r{r}/m{j}/client{i}"), device)
                cache[e] = TR(store.put(w) if store is not None else w, c)
            specs.append((mids[j], cache, sum(mm["counts"])))
        top, deltas = sync_hierarchy_round(specs, top, with_delta=with_delta)
        for j in range(len(rm["mids"])):
            res.append((f"r{r}/m{j}/new", to_cpu(mids[j]), fx.weights(f"r{r}/m{j}/new")))
            if with_delta:
                res.append((f"r{r}/m{j}/delta", to_cpu(deltas[j]), fx.weights(f"r{r}/m{j}/delta")))
        res.append((f"r{r}/top", to_cpu(top), fx.weights(f"r{r}/top")))
        del specs
    return res


class _PRE:
    """Stands in for flame.common.constants.TrainState.PRE (value "pre")."""
    value = "pre"


def run_feddyn(fx, make_opt, device):
    """feddyn/top_aggregator.py:101-107,140,163-165 call pattern (make_golden.feddyn_rounds)."""
    m = fx.meta
    opt = make_opt("feddyn", alpha=m["alpha"])
    cld = to_dev(fx.weights("weights0"), device)
    res = []
    for r, ends in enumerate(m["rounds"]):
        opt.save_state(_PRE, active_ends=m["all_ends"])
        cache = SortedCache()
        for i, (e, c) in enumerate(zip(ends, m["counts"][r])):
            cache[e] = TR(to_dev(fx.weights(f"r{r}/client{i}"), device), c)
        assert list(cache.iterkeys()) == m["orders"][r]
        out = opt.do(deepcopy(cld), cache, total=sum(m["counts"][r]), num_trainers=len(ends))
        assert len(cache) == 0
        cld = opt.cld_model
        res.append((f"r{r}/avg", to_cpu(out), fx.weights(f"r{r}/avg")))
        res.append((f"r{r}/cld", to_cpu(cld), fx.weights(f"r{r}/cld")))
    return res


def run_scaffold(fx, make_opt, device):
    """scaffold/top_aggregator.py:115-126,160,177 call pattern (make_golden.scaffold_rounds)."""
    m = fx.meta
    opt = make_opt("scaffold", k=m["k"])
    opt.save_state(_PRE, dataset_sizes=m["dataset_sizes"])
    weights = to_dev(fx.weights("weights0"), device)
    res = []
    for r, ends in enumerate(m["rounds"]):
        opt.save_state(_PRE, glob_weights=weights)
        cache, control_cache = SortedCache(), SortedCache()
        for i, e in enumerate(ends):
            cache[e] = TR(to_dev(fx.weights(f"r{r}/client{i}"), device), m["dataset_sizes"][e])
            control_cache[e] = TR(to_dev(fx.weights(f"r{r}/control{i}"), device))
        weights = opt.do(deepcopy(weights), cache, total=sum(m["dataset_sizes"][e] for e in ends),
                         num_trainers=len(ends), control_cache=control_cache)
        assert len(cache) == 0 and len(control_cache) == 0
        res.append((f"r{r}/out", to_cpu(weights), fx.weights(f"r{r}/out")))
        res.append((f"r{r}/c_glob", to_cpu(opt.c_glob), fx.weights(f"r{r}/c_glob")))
    return res


class _LocalBias:
    """Duck-typed trainer-side Bias terms (bias.py:34-42) as the top aggregator receives them."""

    def __init__(self, a, b, c, d, val):
        self.a, self.b, self.c, self.d, self.val = a, b, c, d, val


def _bias_terms(opt):
    if hasattr(opt, "bias_terms"):
        return opt.bias_terms()
    b = opt.bias
    return [b.a, b.b, b.c, b.d, b.val, b.sign]


def run_fedgft(fx, make_opt, device):
    """fedgft/top_aggregator.py:52-86 + syncfl aggregate (make_golden.fedgft_rounds):
    do(deepcopy(weights), cache, total=...) then update_bias(dataset_sizes, local_biases)."""
    m = fx.meta
    res = []
    for fair in m["fairs"]:
        opt = make_opt("fedgft", fair=fair, gamma=m["gamma"])
        w = to_dev(fx.weights("weights0"), device)
        for r, ends in enumerate(m["rounds"]):
            tag = f"{fair}/r{r}"
            bm = m["bias"][tag]
            cache = SortedCache()
            for i, (e, c) in enumerate(zip(ends, bm["counts"])):
                cache[e] = TR(to_dev(fx.weights(f"{tag}/client{i}"), device), c)
            assert list(cache.iterkeys()) == bm["order"]
            w = opt.do(deepcopy(w), cache, total=sum(bm["counts"]), num_trainers=len(ends))
            assert len(cache) == 0
            local = {e: _LocalBias(*t) for e, t in zip(ends, bm["local"])}
            opt.update_bias(dataset_sizes={e: bm["sizes"][e] for e in ends}, local_biases=local)
            res.append((f"{tag}/out", to_cpu(w), fx.weights(f"{tag}/out")))
            got = {"bias": torch.tensor(_bias_terms(opt) + [opt.get_bias()], dtype=torch.float64)}
            exp = {"bias": torch.tensor(bm["global"] + [bm["get_bias"]], dtype=torch.float64)}
            res.append((f"{tag}/bias", got, exp))
    return res


BITWISE_FIXTURES = [
    ("fedavg_small.npz", run_fedavg),
    ("fedavg_dtypes.npz", run_fedavg),
    ("fedavg_edge_p1.npz", run_fedavg),
    ("fedavg_edge_p4099.npz", run_fedavg),
    ("fedavg_mnist2.npz", run_fedavg_synth),
    ("fedavg_eager.npz", run_fedavg_eager),
    ("fedavg_edge_none.npz", run_none),
    ("fedbuff_seq_fp32.npz", run_fedbuff_seq),
    ("fedbuff_seq_bf16.npz", run_fedbuff_seq),
    ("fedbuff_none_multi.npz", run_fedbuff_none_multi),
    ("fedavg_subsets.npz", run_fedavg),
    ("fedbuff_subsets.npz", run_fedbuff_subsets),
    ("fedbuff_dtypes.npz", run_fedbuff_dtypes),
    ("downcast.npz", run_downcast),
    ("narrow.npz", run_narrow),
    ("feddyn_rounds.npz", run_feddyn),
    ("feddyn_narrow.npz", run_feddyn),
    ("scaffold_rounds.npz", run_scaffold),
    ("scaffold_narrow.npz", run_scaffold),
    ("fedgft_rounds.npz", run_fedgft),
    ("hier_fedavg_small.npz", run_hier_fedavg),
]
FEDOPT_FIXTURES = ["fedadam_rounds.npz", "fedyogi_rounds.npz", "fedadagrad_rounds.npz", "fedadam_mixed_rounds.npz",
                   "fedyogi_mixed_rounds.npz", "fedadagrad_mixed_rounds.npz"]


def delta_torch(a, b):
    """common/util.py:152-159 restated."""
    return {x: a[x] - b[y] for (x, y) in zip(a, b)}


def rate_fedbuff(version, tres_version):
    return 1 / math.sqrt(1 + version - tres_version)


def fedopt_identical_state_rounds(fx, device):
    """For each adaptive round r >= 1 of a FedOPT fixture, yield the reference's
    state before round r and its expected outputs, so one round can be checked
    elementwise from identical state."""
    m = fx.meta
    for r in range(1, m["rounds"]):
        clients = [to_dev(fx.weights(f"r{r}/client{i}"), device) for i in range(m["n"])]
        counts = m["counts"][r]
        state = {
            "cur": to_dev(fx.weights(f"r{r - 1}/cur"), device),
            "m": to_dev(fx.weights(f"r{r - 1}/m"), device) if f"r{r - 1}/m" in m["keys"] else None,
            "v": to_dev(fx.weights(f"r{r - 1}/v"), device) if f"r{r - 1}/v" in m["keys"] else None,
        }
        exp = {"cur": fx.weights(f"r{r}/cur"), "m": fx.weights(f"r{r}/m"), "v": fx.weights(f"r{r}/v"),
               "avg": fx.weights(f"r{r}/avg")}
        yield r, clients, counts, state, exp


def nonfinite_case(dtype, n=5, P=4099, seed=61):
    """Client updates with NaN, +-inf and values whose weighted sum overflows (a diverged
    trainer): base, clients, counts."""
    g = torch.Generator().manual_seed(seed)
    big = {torch.float32: 3.0e38, torch.bfloat16: 3.0e38, torch.float16: 6.0e4, torch.float64: 1.7e308}[dtype]
    base = torch.randn(P, generator=g, dtype=torch.float64).to(dtype)
    cl = []
    for i in range(n):
        c = (torch.randn(P, generator=g, dtype=torch.float64) * 1e-2).to(dtype)
        c[i::97] = float("nan")
        c[(i + 11)::89] = float("inf")
        c[(i + 23)::83] = -float("inf")
        c[(i + 37)::79] = big            # sums of several of these overflow to inf
        c[(i + 41)::73] = -big
        cl.append(c)
    base[::101] = float("nan")
    base[7::103] = float("inf")
    return base, cl, [100 + 7 * i for i in range(n)]


def assert_same_nonfinite(label, got, exp):
    """Equal where finite or infinite (bitwise), NaN in exactly the same places.  NaN sign /
    payload bits are not pinned: IEEE 754 leaves them open and torch-CPU's depend on the ISA."""
    g = got.detach().cpu().double()
    e = exp.detach().cpu().double()
    gn, en = torch.isnan(g), torch.isnan(e)
    assert torch.equal(gn, en), f"{label}: NaN positions differ ({int((gn ^ en).sum())} elements)"
    assert torch.equal(g[~gn], e[~en]), f"{label}: non-NaN values differ"


# ---------------------------------------------------------------- oracle hierarchies (per-rank stand-ins)
def oracle_hierarchy_round(middles, top_agg=None, *, version, top_weights=None, top_goal=None, with_delta=False,
                           update_middle_weights=True, key_groups=None, after_group=None):
    """flame_amd.optimizer.fedbuff.hierarchy_round restated with the oracle FedBuff, op for op
    as the roles issue it: per middle scale_add (fedbuff.py:101-127) + delta
    (asyncfl/middle_aggregator.py:221-226,246), the top's do per delta (top_aggregator.py:85-92),
    then the top's scale_add."""
    from oracle import oracle as O
    top = O.OracleFedBuff()
    deltas = []
    for i, (w, agg, goal, mv) in enumerate(middles):
        mw = w if update_middle_weights else {k: v.clone() for k, v in w.items()}
        prev = {k: v.clone() for k, v in mw.items()}
        O.OracleFedBuff().scale_add_agg_weights(mw, {k: agg[k] for k in mw}, goal)
        d = {k: mw[k] - prev[k] for k in mw}
        deltas.append(d)
        c = SortedCache()
        c[f"mid{i:05d}"] = TR(d, 1, mv)
        top_agg = top.do(top_agg, c, total=1, version=version)
    if top_weights is not None:
        top.scale_add_agg_weights(top_weights, top_agg, top_goal)
    for gi in range(len(key_groups or ())):
        after_group(gi)
    return top_agg, (deltas if with_delta else None)


def oracle_sync_hierarchy_round(middles, top_weights, *, with_delta=False, update_middle_weights=True,
                                key_groups=None, after_group=None):
    """flame_amd.optimizer.sync_hierarchy.sync_hierarchy_round restated with the oracle FedAvg:
    per middle FedAvg.do(deepcopy(w)) + delta (syncfl/middle_aggregator.py:163-229), the top's
    FedAvg over the deltas with rate total_m / sum (syncfl/top_aggregator.py:122-176)."""
    from oracle import oracle as O
    top_cache, deltas, totals = SortedCache(), [], []
    for i, (w, cache, total) in enumerate(middles):
        new = O.OracleFedAvg().do({k: v.clone() for k, v in w.items()}, cache, total=total)
        d = {k: new[k] - w[k] for k in w}
        if update_middle_weights:
            for k in w:
                w[k].copy_(new[k])
        deltas.append(d)
        top_cache[f"mid{i:05d}"] = TR(d, total)
        totals.append(total)
    O.OracleFedAvg().do(top_weights, top_cache, total=sum(totals))
    for gi in range(len(key_groups or ())):
        after_group(gi)
    return top_weights, (deltas if with_delta else None)


def run_nonfinite(fx, make_opt, device):
    """nonfinite.npz: per float dtype, FedAvg and FedBuff (+ scale_add) over a diverged
    trainer's updates; yields (label, got, expected) compared with assert_same_nonfinite."""
    m = fx.meta
    for tag in m["float_dtypes"]:
        base = fx.weights(f"{tag}/base")["w"]
        cl = [fx.weights(f"{tag}/client{i}")["w"] for i in range(m["n"])]
        cache = SortedCache()
        for i, c in enumerate(cl):
            cache[f"e{i}"] = TR({"w": c.to(device)}, m["counts"][i])
        got = make_opt("fedavg").do({"w": base.clone().to(device)}, cache, total=sum(m["counts"]))
        yield f"{tag}/fedavg", got["w"], fx.weights(f"{tag}/fedavg")["w"]
        fb, agg = make_opt("fedbuff"), None
        for i, c in enumerate(cl):
            one = SortedCache()
            one["a"] = TR({"w": c.to(device)}, 1, m["round"] - m["stale"][i])
            agg = fb.do(agg, one, total=1, version=m["round"])
        yield f"{tag}/fedbuff_agg", to_cpu(agg)["w"], fx.weights(f"{tag}/fedbuff_agg")["w"]
        w = {"w": base.clone().to(device)}
        fb.scale_add_agg_weights(w, agg, m["n"])
        yield f"{tag}/fedbuff_out", w["w"], fx.weights(f"{tag}/fedbuff_out")["w"]
