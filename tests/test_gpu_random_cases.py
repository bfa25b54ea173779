"""Randomised differential cases: the drop-in optimizers on the GPU vs the oracle, on models and
rounds drawn from a seeded generator -- the combinations the hand-written tests do not pin one by
one.  Each case draws: the optimizer (FedAvg, FedBuff do-per-arrival + scale_add with or without
the middle delta, FedAdam / FedYogi / FedAdaGrad over three rounds, and the eager callers: FedAvg
with a running total per arrival, deferred or not, and FedOPT whose current aliases the base,
eager_syncfl/top_aggregator.py:36-90), 1-4 keys whose dtypes and
sizes mix (0, 1, chunk boundaries +-1, up to 300k elements; FedAvg adds int64 / int32 buffers),
1-150 clients, and where the updates live (separate HBM tensors, tiled UpdateSlab slots, or views
one element off their allocation's alignment).  FedAvg / FedBuff: every element bitwise
(fedavg.py:89-104, fedbuff.py:89-157, including the None-start quirk when a first call carries
several entries); FedOPT: the first round bitwise, the adaptive rounds within the SURVEY §8(c)
contract (fedopt.py:102-129).
"""
import os

import numpy as np
import pytest
import torch

import scenarios as S

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
SORTS = ["fedavg", "fedbuff", "fedadam", "fedyogi", "fedadagrad", "fedavg_eager", "fedopt_eager"]
# A soak run draws more, different cases: FLAME_RANDOM_SCALE multiplies every case count and
# FLAME_RANDOM_SEED_OFFSET moves every seed range (defaults: the suite's own 391 cases).
SCALE = max(1, int(os.environ.get("FLAME_RANDOM_SCALE", "1")))
SEED_OFFSET = int(os.environ.get("FLAME_RANDOM_SEED_OFFSET", "0"))
N_CASES = 7 * 40 * SCALE
FLOATS = [torch.float32, torch.bfloat16, torch.float16, torch.float64]
INTS = [torch.int64, torch.int32]


@pytest.fixture(scope="module", autouse=True)
def _native_loaded():
    from flame_amd import _native
    _native.lib()
    assert torch.cuda.is_available()
    torch.empty(1, device=DEV)


def _oracle():
    from oracle import oracle as O
    return O


def _draw_size(rng, dtype):
    from flame_amd import engine
    c = engine.chunk_elems(engine.dtype_code(dtype))
    pick = rng.integers(0, 8)
    return int([0, 1, 7, c - 1, c, c + 1, 2 * c + 3, rng.integers(1, 300_000)][pick])


def _draw_case(i):
    rng = np.random.default_rng(7_000 + SEED_OFFSET + i)
    sort = SORTS[i % len(SORTS)]
    n_keys = int(rng.integers(1, 5))
    keys = []
    for k in range(n_keys):
        if sort in ("fedavg", "fedavg_eager"):
            dt = FLOATS[rng.integers(0, 4)] if rng.random() < 0.8 else INTS[rng.integers(0, 2)]
        elif sort == "fedbuff":
            dt = FLOATS[rng.integers(0, 4)]
        else:
            dt = torch.float32
        keys.append((f"k{k}", dt, _draw_size(rng, dt)))
    placement = ["hbm", "slab", "views"][rng.integers(0, 3)]
    if placement == "slab" and any(s == 0 for _, _, s in keys):
        placement = "hbm"
    if rng.random() < 0.1:          # now and then one big key (fewer clients)
        dt = keys[0][1]
        keys[0] = (keys[0][0], dt, int(rng.integers(1_000_000, 3_000_000)))
    total_elems = max(1, sum(s for _, _, s in keys))
    n = int(rng.integers(1, 151 if not sort.endswith("eager") else 40))
    n = max(1, min(n, 6_000_000 // total_elems))
    return rng, sort, keys, placement, n


def _rand(g, shape, dtype, scale):
    if dtype.is_floating_point:
        return (torch.randn(shape, generator=g, dtype=torch.float64) * scale).to(dtype)
    return torch.randint(-50, 50, shape, generator=g, dtype=dtype)


class _Placer:
    """Puts a client's update on the device the way the case says."""

    def __init__(self, placement, keys, n):
        from flame_amd.slab import UpdateSlab
        self.placement = placement
        self.slab = None
        if placement == "slab":
            tmpl = {k: torch.zeros(s, dtype=dt) for k, dt, s in keys}
            self.slab = UpdateSlab(tmpl, capacity=n, device=DEV)

    def put(self, w):
        if self.placement == "slab":
            return self.slab.put({k: v.to(DEV) for k, v in w.items()})
        if self.placement == "views":
            out = {}
            for k, v in w.items():
                buf = torch.empty(v.numel() + 1, dtype=v.dtype, device=DEV)
                buf[1:].copy_(v.to(DEV))
                out[k] = buf[1:]
            return out
        return {k: v.to(DEV) for k, v in w.items()}


def _run_fedavg(rng, keys, placement, n, label):
    from flame_amd.optimizers import optimizer_provider
    O = _oracle()
    g = torch.Generator().manual_seed(int(rng.integers(1 << 31)))
    base = {k: _rand(g, (s,), dt, 1.0) for k, dt, s in keys}
    ups = [{k: _rand(g, (s,), dt, 1e-2) for k, dt, s in keys} for _ in range(n)]
    counts = [int(c) for c in rng.integers(1, 1000, n)]
    total = sum(counts)
    P = _Placer(placement, keys, n)
    cache = S.SortedCache()
    for i in range(n):
        cache[f"{i:04d}"] = S.TR(P.put(ups[i]), counts[i])
    out = optimizer_provider.get("fedavg").do(S.to_dev(base, DEV), cache, total=total)
    exp = {k: v.clone() for k, v in base.items()}
    for k in exp:
        O.reduce_tensor(exp[k], [u[k] for u in ups], [c / total for c in counts])
    S.assert_bitwise(label, out, exp)


def _run_fedbuff(rng, keys, placement, n, label):
    from flame_amd.optimizers import optimizer_provider
    O = _oracle()
    g = torch.Generator().manual_seed(int(rng.integers(1 << 31)))
    version = 20
    P = _Placer(placement, keys, n)
    amd, ora = optimizer_provider.get("fedbuff"), O.OracleFedBuff()
    aa = ao = None
    i = 0
    while i < n:
        m = int(min(n - i, rng.integers(1, 4)))        # entries in this do() call
        ca, co = S.SortedCache(), S.SortedCache()
        for j in range(m):
            u = {k: _rand(g, (s,), dt, 1e-2) for k, dt, s in keys}
            stale = int(rng.integers(0, 4))
            count = int(rng.integers(1, 50))
            ca[f"{i + j:04d}"] = S.TR(P.put(u), count, version - stale)
            co[f"{i + j:04d}"] = S.TR(u, count, version - stale)
        aa = amd.do(aa, ca, total=m, version=version)
        ao = ora.do(ao, co, total=m, version=version)
        i += m
    goal = n
    model = {k: _rand(g, (s,), dt, 1.0) for k, dt, s in keys}
    dev_model = S.to_dev(model, DEV)
    want_delta = bool(rng.integers(0, 2))
    exp_delta = {}
    for k in model:
        d = O.scale_add_tensor(model[k], ao[k], goal, want_delta=want_delta)
        if want_delta:
            exp_delta[k] = d
    if want_delta:
        _, got_delta = amd.scale_add_agg_weights_with_delta(dev_model, aa, goal)
        S.assert_bitwise(label + "/delta", got_delta, exp_delta)
    else:
        amd.scale_add_agg_weights(dev_model, aa, goal)
    S.assert_bitwise(label + "/model", dev_model, model)


def _run_fedopt(rng, sort, keys, placement, n, label):
    from flame_amd.optimizers import optimizer_provider
    O = _oracle()
    g = torch.Generator().manual_seed(int(rng.integers(1 << 31)))
    w0 = {k: _rand(g, (s,), dt, 1.0) for k, dt, s in keys}
    P = _Placer(placement, keys, 3 * n)      # three rounds of slots, however soon they return
    amd, ora = optimizer_provider.get(sort), O.OracleFedOPT(sort)
    wa, wo = S.to_dev(w0, DEV), {k: v.clone() for k, v in w0.items()}
    for r in range(3):
        ups = [{k: _rand(g, (s,), dt, 1e-2) for k, dt, s in keys} for _ in range(n)]
        counts = [int(c) for c in rng.integers(1, 1000, n)]
        ca, co = S.SortedCache(), S.SortedCache()
        for i in range(n):
            ca[f"{i:04d}"] = S.TR(P.put(ups[i]), counts[i])
            co[f"{i:04d}"] = S.TR(ups[i], counts[i])
        wa = amd.do({k: v.clone() for k, v in wa.items()}, ca, total=sum(counts))
        wo = ora.do({k: v.clone() for k, v in wo.items()}, co, total=sum(counts))
        if r == 0:
            S.assert_bitwise(f"{label}/r0", wa, wo)
        else:
            S.assert_close_fedopt(f"{label}/r{r}", S.to_cpu(wa), wo, elementwise=r == 1)
        del ca


def _run_fedavg_eager(rng, keys, placement, n, label):
    """One do() per arrival with the running total (eager_syncfl/top_aggregator.py:36-90)."""
    from flame_amd.optimizers import optimizer_provider
    O = _oracle()
    g = torch.Generator().manual_seed(int(rng.integers(1 << 31)))
    defer = bool(rng.integers(0, 2))
    base = {k: _rand(g, (s,), dt, 1.0) for k, dt, s in keys}
    dev_base = S.to_dev(base, DEV)
    P = _Placer(placement, keys, n)
    amd, ora = optimizer_provider.get("fedavg", defer=defer), O.OracleFedAvg()
    ca, co = S.SortedCache(), S.SortedCache()
    total = 0
    check_at = int(rng.integers(0, n))
    for i in range(n):
        u = {k: _rand(g, (s,), dt, 1e-2) for k, dt, s in keys}
        c = int(rng.integers(1, 1000))
        total += c
        ca[f"{i:04d}"] = S.TR(P.put(u), c)
        co[f"{i:04d}"] = S.TR(u, c)
        out = amd.do(dev_base, ca, total=total, num_trainers=n)
        ora.do(base, co, total=total)
        if i == check_at or i == n - 1:
            S.assert_bitwise(f"{label}/defer={defer}/after{i}", {k: v for k, v in S.to_cpu(out).items()}, base)


def _run_fedopt_eager(rng, keys, placement, n, label):
    """The eager top's FedOPT: per round base = deepcopy(weights), then do(base, cache,
    total=running) per arrival -- current aliases base after the first call."""
    from copy import deepcopy
    from flame_amd.optimizers import optimizer_provider
    O = _oracle()
    g = torch.Generator().manual_seed(int(rng.integers(1 << 31)))
    sort = ["fedadam", "fedyogi", "fedadagrad"][rng.integers(0, 3)]
    w0 = {k: _rand(g, (s,), dt, 1.0) for k, dt, s in keys}
    P = _Placer(placement, keys, 2 * n)
    # defer=True: the round's calls run as one flame_fedopt_chain launch when the result is read
    defer = bool(g.initial_seed() % 2)
    label += f" defer={defer}"
    amd, ora = optimizer_provider.get(sort, defer=defer), O.OracleFedOPT(sort)
    wa, wo = S.to_dev(w0, DEV), {k: v.clone() for k, v in w0.items()}
    for r in range(2):
        ba, bo = deepcopy(wa), deepcopy(wo)
        ca, co = S.SortedCache(), S.SortedCache()
        total = 0
        for i in range(n):
            u = {k: _rand(g, (s,), dt, 1e-2) for k, dt, s in keys}
            c = int(rng.integers(1, 1000))
            total += c
            ca[f"r{r}e{i:04d}"] = S.TR(P.put(u), c)
            co[f"r{r}e{i:04d}"] = S.TR(u, c)
            oa = amd.do(ba, ca, total=total, num_trainers=n)
            oo = ora.do(bo, co, total=total)
        S.assert_close_fedopt(f"{label}/{sort}/r{r}", S.to_cpu(oa), oo, elementwise=r == 0)
        wa, wo = oa, oo


@pytest.mark.oracle
@pytest.mark.parametrize("case", range(N_CASES))
def test_random_case_vs_oracle(case):
    rng, sort, keys, placement, n = _draw_case(case)
    label = (f"case {case}: {sort} {placement} n={n} keys=" +
             ",".join(f"{k}:{str(dt).replace('torch.', '')}[{s}]" for k, dt, s in keys))
    if sort == "fedavg":
        _run_fedavg(rng, keys, placement, n, label)
    elif sort == "fedavg_eager":
        _run_fedavg_eager(rng, keys, placement, n, label)
    elif sort == "fedopt_eager":
        _run_fedopt_eager(rng, keys, placement, n, label)
    elif sort == "fedbuff":
        _run_fedbuff(rng, keys, placement, n, label)
    else:
        _run_fedopt(rng, sort, keys, placement, n, label)


def test_random_cases_cover_every_draw():
    """The seeded draw reaches every optimizer, placement, float dtype and a zero-size key."""
    seen = set()
    for i in range(N_CASES):
        _, sort, keys, placement, n = _draw_case(i)
        seen.add(sort)
        seen.add(placement)
        for _, dt, s in keys:
            seen.add(dt)
            if s == 0:
                seen.add("empty")
    for want in (*SORTS, "hbm", "slab", "views", "empty", *FLOATS):
        assert want in seen, want


# ---------------------------------------------------------------- co-located hierarchies
N_HIER = 60 * SCALE
HFLOATS = [torch.float32, torch.bfloat16, torch.float16]


def _draw_hier(i):
    rng = np.random.default_rng(9_000 + SEED_OFFSET + i)
    mode = "async" if i % 2 == 0 else "sync"
    keys = []
    for k in range(int(rng.integers(1, 4))):
        dt = HFLOATS[rng.integers(0, 3)]
        keys.append((f"k{k}", dt, _draw_size(rng, dt)))
    M = int(rng.integers(1, 25))
    arrivals = [int(rng.integers(1, 7)) for _ in range(M)]        # ragged middles
    per_elem = max(1, sum(s for _, _, s in keys))
    while sum(arrivals) * per_elem > 4_000_000 and max(arrivals) > 1:
        arrivals = [max(1, a // 2) for a in arrivals]
    placement = ["slab", "tensors", "mixed"][rng.integers(0, 3)]
    if any(s == 0 for _, _, s in keys):
        placement = "tensors"
    return rng, mode, keys, arrivals, placement


def _run_hier_async(rng, keys, arrivals, placement, label):
    from flame_amd.optimizer.fedbuff import hierarchy_round
    from flame_amd.optimizers import optimizer_provider
    from flame_amd.slab import UpdateSlab
    O = _oracle()
    g = torch.Generator().manual_seed(int(rng.integers(1 << 31)))
    M, rnd = len(arrivals), 12
    mk = lambda scale: {k: _rand(g, (s,), dt, scale) for k, dt, s in keys}       # noqa: E731
    ups = [[mk(1e-2) for _ in range(a)] for a in arrivals]
    vers = [[rnd - int(rng.integers(0, 4)) for _ in range(a)] for a in arrivals]
    mid0 = [mk(1.0) for _ in range(M)]
    goals = [int(rng.integers(1, 9)) for _ in range(M)]
    mid_ver = [rnd - int(rng.integers(0, 3)) for _ in range(M)]
    top_start = bool(rng.integers(0, 2))
    top_prev = mk(1e-3)
    top_w0 = mk(1.0) if rng.integers(0, 2) else None
    top_goal = int(rng.integers(1, 10))
    with_delta = bool(rng.integers(0, 2))
    update_mids = bool(rng.integers(0, 2))
    slab = (UpdateSlab({k: torch.empty(s, dtype=dt) for k, dt, s in keys}, capacity=sum(arrivals), device=DEV)
            if placement != "tensors" else None)
    aggs = []
    for m in range(M):
        opt, agg = optimizer_provider.get("fedbuff"), None
        for t in range(arrivals[m]):
            w = S.to_dev(ups[m][t], DEV)
            in_slab = slab is not None and (placement == "slab" or (m + t) % 2 == 0)
            c = S.SortedCache()
            c["a"] = S.TR(slab.put(w) if in_slab else w, 1, vers[m][t])
            agg = opt.do(agg, c, total=1, version=rnd)
        aggs.append(agg)
    mids = [S.to_dev(w, DEV) for w in mid0]
    tw = S.to_dev(top_w0, DEV) if top_w0 is not None else None
    ta = S.to_dev(top_prev, DEV) if top_start else None
    agg, deltas = hierarchy_round([(mids[m], aggs[m], goals[m], mid_ver[m]) for m in range(M)], ta, version=rnd,
                                  top_weights=tw, top_goal=top_goal, with_delta=with_delta,
                                  update_middle_weights=update_mids)
    # oracle
    oaggs = []
    for m in range(M):
        mo, ao = O.OracleFedBuff(), None
        for t in range(arrivals[m]):
            c = S.SortedCache()
            c["a"] = S.TR({k: v.clone() for k, v in ups[m][t].items()}, 1, vers[m][t])
            ao = mo.do(ao, c, total=1, version=rnd)
        oaggs.append(ao)
    omids = [{k: v.clone() for k, v in w.items()} for w in mid0]
    otw = {k: v.clone() for k, v in top_w0.items()} if top_w0 is not None else None
    oagg, odeltas = S.oracle_hierarchy_round(
        [(omids[m], oaggs[m], goals[m], mid_ver[m]) for m in range(M)],
        {k: v.clone() for k, v in top_prev.items()} if top_start else None, version=rnd, top_weights=otw,
        top_goal=top_goal, with_delta=with_delta, update_middle_weights=update_mids)
    label += f" top_start={top_start} top_w={top_w0 is not None} delta={with_delta} update={update_mids}"
    S.assert_bitwise(label + "/top agg", S.to_cpu(dict(agg)), oagg)
    for m in range(M):
        S.assert_bitwise(f"{label}/mid{m}", S.to_cpu(mids[m]), omids[m])
        if with_delta:
            S.assert_bitwise(f"{label}/delta{m}", S.to_cpu(deltas[m]), odeltas[m])
    if otw is not None:
        S.assert_bitwise(label + "/top w", S.to_cpu(tw), otw)


def _run_hier_sync(rng, keys, arrivals, placement, label):
    from flame_amd.optimizer.sync_hierarchy import sync_hierarchy_round
    from flame_amd.slab import UpdateSlab
    g = torch.Generator().manual_seed(int(rng.integers(1 << 31)))
    M = len(arrivals)
    mk = lambda scale: {k: _rand(g, (s,), dt, scale) for k, dt, s in keys}       # noqa: E731
    ups = [[mk(1e-2) for _ in range(a)] for a in arrivals]
    counts = [[int(rng.integers(1, 500)) for _ in range(a)] for a in arrivals]
    mid0 = [mk(1.0) for _ in range(M)]
    top0 = mk(1.0)
    with_delta = bool(rng.integers(0, 2))
    update_mids = bool(rng.integers(0, 2))
    slab = (UpdateSlab({k: torch.empty(s, dtype=dt) for k, dt, s in keys}, capacity=sum(arrivals), device=DEV)
            if placement != "tensors" else None)
    mids, tops = [S.to_dev(w, DEV) for w in mid0], S.to_dev(top0, DEV)
    middles, omiddles = [], []
    omids = [{k: v.clone() for k, v in w.items()} for w in mid0]
    for m in range(M):
        c, oc = S.SortedCache(), S.SortedCache()
        for t in range(arrivals[m]):
            w = S.to_dev(ups[m][t], DEV)
            in_slab = slab is not None and (placement == "slab" or (m + t) % 2 == 0)
            c[f"e{t:03d}"] = S.TR(slab.put(w) if in_slab else w, counts[m][t])
            oc[f"e{t:03d}"] = S.TR(ups[m][t], counts[m][t])
        middles.append((mids[m], c, sum(counts[m])))
        omiddles.append((omids[m], oc, sum(counts[m])))
    _, deltas = sync_hierarchy_round(middles, tops, with_delta=with_delta, update_middle_weights=update_mids)
    otop = {k: v.clone() for k, v in top0.items()}
    _, odeltas = S.oracle_sync_hierarchy_round(omiddles, otop, with_delta=with_delta,
                                               update_middle_weights=update_mids)
    label += f" delta={with_delta} update={update_mids}"
    S.assert_bitwise(label + "/top", S.to_cpu(tops), otop)
    for m in range(M):
        S.assert_bitwise(f"{label}/mid{m}", S.to_cpu(mids[m]), omids[m])
        if with_delta:
            S.assert_bitwise(f"{label}/delta{m}", S.to_cpu(deltas[m]), odeltas[m])


@pytest.mark.oracle
@pytest.mark.parametrize("case", range(N_HIER))
def test_random_hierarchy_vs_oracle(case, monkeypatch):
    """The co-located hierarchies (flame_hier_fedbuff: async FedBuff middles + top, and the
    synchronous FedAvg one) on drawn shapes: 1-24 middles with 1-6 arrivals each (ragged), mixed
    key dtypes, slab / tensor / mixed arrivals, an existing or None top aggregate, top weights or
    not, deltas or not, read-only or updated middles, the kernel-argument or the device-table
    launch -- every output bitwise against the oracle's per-role op sequence."""
    from flame_amd import engine
    rng, mode, keys, arrivals, placement = _draw_hier(case)
    if rng.integers(0, 2):
        monkeypatch.setattr(engine, "ARGMETA", False)
    label = (f"hier case {case}: {mode} {placement} M={len(arrivals)} arrivals={arrivals} "
             f"argmeta={engine.ARGMETA} keys=" + ",".join(f"{k}:{str(dt).replace('torch.', '')}[{s}]"
                                                            for k, dt, s in keys))
    if mode == "async":
        _run_hier_async(rng, keys, arrivals, placement, label)
    else:
        _run_hier_sync(rng, keys, arrivals, placement, label)


# ---------------------------------------------------------------- FedDyn / SCAFFOLD
N_STATEFUL = 30 * SCALE


def _draw_model(rng, g):
    keys = {}
    for k in range(int(rng.integers(1, 5))):
        dt = [torch.float32, torch.bfloat16, torch.float16, torch.float64][rng.integers(0, 4)]
        keys[f"k{k}"] = _rand(g, (_draw_size(rng, dt) or 1,), dt, 1.0)
    if rng.integers(0, 2):
        keys["nbt"] = torch.tensor(int(rng.integers(0, 9)), dtype=torch.int64)
    return keys


def _update(g, tmpl, i, scale=1e-2):
    return {k: _rand(g, v.shape, v.dtype, scale) if v.is_floating_point() else torch.tensor(i, dtype=v.dtype)
            for k, v in tmpl.items()}


def _run_feddyn(rng, label):
    from flame_amd.optimizers import optimizer_provider
    from flame_amd.slab import UpdateSlab
    O = _oracle()
    g = torch.Generator().manual_seed(int(rng.integers(1 << 31)))
    tmpl = _draw_model(rng, g)
    per = sum(v.numel() for v in tmpl.values())
    n_ends = int(max(2, min(rng.integers(2, 41), 3_000_000 // per)))
    ends = [f"e{i:02d}" for i in range(n_ends)]
    active = list(ends) if rng.integers(0, 2) else [ends[i] for i in rng.permutation(n_ends)]
    history = ["rows", "pingpong", "pingpong_rows"][rng.integers(0, 3)]
    alpha = float(rng.choice([0.01, 0.1, 0.5]))
    placement = ["hbm", "slab"][rng.integers(0, 2)]
    label += f" ends={n_ends} history={history} alpha={alpha} {placement} order={'cache' if active == ends else 'other'}"
    slab = UpdateSlab(tmpl, capacity=2 * n_ends, device=DEV) if placement == "slab" else None
    amd = optimizer_provider.get("feddyn", alpha=alpha, history=history)
    ora = O.OracleFedDyn(alpha=alpha)
    wa, wo = S.to_dev(tmpl, DEV), {k: v.clone() for k, v in tmpl.items()}
    for r in range(int(rng.integers(2, 5))):
        amd.save_state(S._PRE, active_ends=active)
        ora.save_state(S._PRE, active_ends=active)
        part = [e for e in ends if rng.random() < 0.7] or ends[:1]
        if rng.random() < 0.2:
            part = part + ["zz"]                     # an end the channel does not list
        ca, co = S.SortedCache(), S.SortedCache()
        counts = [int(rng.integers(1, 300)) for _ in part]
        for i, (e, c) in enumerate(zip(part, counts)):
            u = _update(g, tmpl, 10 * r + i)
            du = S.to_dev(u, DEV)
            ca[e] = S.TR(slab.put(du) if slab is not None else du, c)
            co[e] = S.TR(u, c)
        a = amd.do({k: v.clone() for k, v in wa.items()}, ca, total=sum(counts))
        o = ora.do({k: v.clone() for k, v in wo.items()}, co, total=sum(counts))
        S.assert_bitwise(f"{label}/r{r}/avg", S.to_cpu(a), o)
        S.assert_bitwise(f"{label}/r{r}/cld", S.to_cpu(amd.cld_model), ora.cld_model)
        wa, wo = amd.cld_model, ora.cld_model
        del ca, co
    for e, h in ora.local_param_dict.items():
        if h is not None:
            S.assert_bitwise(f"{label}/hist/{e}", S.to_cpu({k: amd.local_param_dict[e][k] for k in h}), h)


def _run_scaffold(rng, label):
    from flame_amd.optimizers import optimizer_provider
    O = _oracle()
    g = torch.Generator().manual_seed(int(rng.integers(1 << 31)))
    tmpl = _draw_model(rng, g)
    per = sum(v.numel() for v in tmpl.values())
    n_ends = int(max(2, min(rng.integers(2, 41), 3_000_000 // per)))
    ends = [f"t{i:02d}" for i in range(n_ends)]
    sizes = {e: int(rng.integers(1, 1000)) for e in ends}
    k = int(rng.integers(1, 6))
    label += f" ends={n_ends} k={k}"
    amd, ora = optimizer_provider.get("scaffold", k=k), O.OracleScaffold(k=k)
    for o in (amd, ora):
        o.save_state(S._PRE, dataset_sizes=sizes)
    wa, wo = S.to_dev(tmpl, DEV), {kk: v.clone() for kk, v in tmpl.items()}
    for r in range(int(rng.integers(2, 4))):
        amd.save_state(S._PRE, glob_weights=wa)
        ora.save_state(S._PRE, glob_weights=wo)
        part = [e for e in ends if rng.random() < 0.6] or ends[:1]
        ws = [_update(g, tmpl, r + i) for i in range(len(part))]
        cs = [_update(g, tmpl, 0, 1e-3) for _ in part]
        for i, c in enumerate(cs):
            if "nbt" in c:
                c["nbt"] = torch.tensor(1.25 * (i + 1) + r)     # an int buffer's control variate is fp32
        ca, cca, co, cco = S.SortedCache(), S.SortedCache(), S.SortedCache(), S.SortedCache()
        for e, w, c in zip(part, ws, cs):
            ca[e] = S.TR(S.to_dev(w, DEV), sizes[e])
            cca[e] = S.TR(S.to_dev(c, DEV))
            co[e] = S.TR(w, sizes[e])
            cco[e] = S.TR(c)
        total = sum(sizes[e] for e in part)
        wa = amd.do({kk: v.clone() for kk, v in wa.items()}, ca, total=total, control_cache=cca)
        wo = ora.do({kk: v.clone() for kk, v in wo.items()}, co, total=total, control_cache=cco)
        S.assert_bitwise(f"{label}/r{r}/out", S.to_cpu(wa), wo)
        S.assert_bitwise(f"{label}/r{r}/c_glob", S.to_cpu(amd.c_glob), ora.c_glob)


@pytest.mark.oracle
@pytest.mark.parametrize("case", range(N_STATEFUL))
def test_random_stateful_vs_oracle(case):
    """FedDyn (partial participation, ends leaving and returning, an unlisted end, the channel's
    order equal to the cache's or not, in-place / ping-pong / ping-pong-rows histories, HBM or
    slab updates; feddyn.py:70-139) and SCAFFOLD (random subsets, k, an int buffer with an fp32
    control variate; scaffold.py:82-150) on drawn models, every output and state bitwise."""
    rng = np.random.default_rng(11_000 + SEED_OFFSET + case)
    label = f"stateful case {case}"
    if case % 2 == 0:
        _run_feddyn(rng, label + " feddyn")
    else:
        _run_scaffold(rng, label + " scaffold")


# ---------------------------------------------------------------- 16-bit eager FedOPT, deferred
N_EAGER16 = 20 * SCALE


@pytest.mark.parametrize("case", range(N_EAGER16))
def test_random_eager_fedopt_16bit_defer_equals_per_call(case):
    """bf16 / fp16 (and mixed) eager FedOPT rounds: FedOPT(defer=True) -- one flame_fedopt_chain
    launch per dtype per round -- against one fused launch per call, bitwise for base, every
    round's current, m_t and v_t (the oracle tests hold 16-bit keys bitwise to the reference's
    torch-CPU op sequence; here the two GPU paths are held to each other)."""
    from copy import deepcopy
    from flame_amd.optimizers import optimizer_provider
    rng = np.random.default_rng(13_000 + SEED_OFFSET + case)
    keys = []
    for k in range(int(rng.integers(1, 4))):
        dt = [torch.bfloat16, torch.float16, torch.float32][rng.integers(0, 3)] if k else \
            [torch.bfloat16, torch.float16][rng.integers(0, 2)]
        keys.append((f"k{k}", dt, _draw_size(rng, dt) or 1))
    placement = ["hbm", "slab", "views"][rng.integers(0, 3)]
    n = int(rng.integers(2, 30))
    sort = ["fedadam", "fedyogi", "fedadagrad"][rng.integers(0, 3)]
    seed = int(rng.integers(1 << 31))
    counts = [int(c) for c in rng.integers(1, 1000, 2 * n)]
    label = (f"eager16 case {case}: {sort} {placement} n={n} keys=" +
             ",".join(f"{k}:{str(dt).replace('torch.', '')}[{s}]" for k, dt, s in keys))

    def run(defer):
        g = torch.Generator().manual_seed(seed)
        w = S.to_dev({k: _rand(g, (s,), dt, 1.0) for k, dt, s in keys}, DEV)
        P = _Placer(placement, keys, 2 * n)
        opt = optimizer_provider.get(sort, defer=defer)
        res = []
        for r in range(2):
            base = deepcopy(w)
            cache = S.SortedCache()
            total = 0
            for i in range(n):
                u = {k: _rand(g, (s,), dt, 1e-2) for k, dt, s in keys}
                total += counts[r * n + i]
                cache[f"r{r}e{i:03d}"] = S.TR(P.put(u), counts[r * n + i])
                out = opt.do(base, cache, total=total)
            w = out
            cur = S.to_cpu(dict(out))
            res.append((S.to_cpu(base), cur, S.to_cpu(opt.m_t) if opt.m_t is not None else {},
                        S.to_cpu(opt.v_t) if opt.v_t is not None else {}))
        return res

    for r, (a, b) in enumerate(zip(run(True), run(False))):
        for lbl, x, y in zip(("base", "current", "m_t", "v_t"), a, b):
            S.assert_bitwise(f"{label}/r{r}/{lbl}", x, y)
