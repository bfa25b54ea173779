"""GPU parity: the HIP path (through the C ABI) vs the golden vectors and the oracle.

Bitwise for FedAvg / FedBuff in every dtype; FedOPT within the SURVEY §8(c)
tolerance (elementwise rel <= 1e-6 where |ref| >= 1e-6*max|ref|, rel-L2 <= 1e-6),
and bitwise wherever only FedAvg arithmetic has happened.
"""
import concurrent.futures
import math

import numpy as np
import pytest
import torch

import scenarios as S

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _native_loaded():
    from flame_amd import _native
    _native.lib()  # fail loudly if the HIP library is missing
    assert torch.cuda.is_available()
    torch.empty(1, device=DEV)   # torch's HIP context: is_pinned() of registered memory needs it


def make_amd(sort, **kw):
    from flame_amd.optimizers import optimizer_provider
    return optimizer_provider.get(sort, **kw)


# ------------------------------------------------------------------ golden vectors
@pytest.mark.oracle
@pytest.mark.parametrize("name,driver", S.BITWISE_FIXTURES, ids=[n for n, _ in S.BITWISE_FIXTURES])
def test_golden_bitwise(golden, name, driver):
    for label, got, exp in driver(golden(name), make_amd, DEV):
        S.assert_bitwise(f"{name}:{label}", got, exp)


@pytest.mark.oracle
@pytest.mark.parametrize("name", S.FEDOPT_FIXTURES)
def test_golden_fedopt(golden, name):
    for label, got, exp in S.run_fedopt(golden(name), make_amd, DEV):
        rnd = int(label.split("/")[0][1:])
        if label in ("r0/cur", "r0/avg", "r1/avg"):
            S.assert_bitwise(f"{name}:{label}", got, exp)
        else:
            # rounds >= 2 start from state that already differs by sqrt ulps: rel-L2 contract
            S.assert_close_fedopt(f"{name}:{label}", got, exp, elementwise=rnd <= 1)


@pytest.mark.oracle
@pytest.mark.parametrize("name", S.FEDOPT_FIXTURES)
def test_golden_fedopt_single_round_elementwise(golden, name):
    """Each adaptive round from the reference's own state: elementwise 1e-6 (avg bitwise)."""
    fx = golden(name)
    m = fx.meta
    for r, clients, counts, state, exp in S.fedopt_identical_state_rounds(fx, DEV):
        opt = make_amd(m["sort"], beta_1=m["beta_1"], beta_2=m["beta_2"], eta=m["eta"], tau=m["tau"])
        opt.current_weights = state["cur"]
        opt.m_t, opt.v_t = state["m"], state["v"]
        cache = S.SortedCache()
        for i, (w, c) in enumerate(zip(clients, counts)):
            cache[f"{i:03d}"] = S.TR(w, c)
        out = opt.do({k: v.clone() for k, v in state["cur"].items()}, cache, total=sum(counts))
        S.assert_bitwise(f"{name}:r{r}/avg", S.to_cpu(opt.agg_weights), exp["avg"])
        for key in ("cur", "m", "v"):
            got = out if key == "cur" else getattr(opt, key + "_t")
            S.assert_close_fedopt(f"{name}:r{r}/{key}", S.to_cpu(got), exp[key])


@pytest.mark.oracle
@pytest.mark.parametrize("name", S.FEDOPT_EAGER_FIXTURES)
def test_golden_fedopt_eager(golden, name):
    """FedAdam / FedYogi driven by the eager top aggregator (same base object every arrival):
    the key whose current_weights aliases base takes d = 0 as the reference does."""
    S.check_fedopt_eager(S.run_fedopt_eager(golden(name), make_amd, DEV))


@pytest.mark.oracle
def test_golden_feddyn_pingpong(golden):
    """FedDyn with ping-pong tiled history stores == the reference fixture, bitwise."""
    def make(sort, **kw):
        return make_amd(sort, history="pingpong", **kw)
    for label, got, exp in S.run_feddyn(golden("feddyn_rounds.npz"), make, DEV):
        S.assert_bitwise(f"feddyn_pingpong:{label}", got, exp)


@pytest.mark.oracle
@pytest.mark.parametrize("name", S.HIER_FIXTURES)
def test_golden_hier_torch_delta(golden, name):
    for label, got, exp in S.run_hier(golden(name), make_amd, DEV, S.delta_torch):
        S.assert_bitwise(f"{name}:{label}", got, exp)


@pytest.mark.oracle
@pytest.mark.parametrize("name", S.HIER_FIXTURES)
def test_golden_hier_fused_delta(golden, name):
    """Middle aggregator using the fused scale_add+delta kernel."""
    fx = golden(name)
    m = fx.meta
    rnd = m["round"]
    mids, arr, _ = S.hier_shape(m)
    top_w0 = fx.weights("top_w0")
    for mid in range(mids):
        opt = make_amd("fedbuff")
        mid_w = S.to_dev(top_w0, DEV)
        agg = None
        for t in range(arr):
            c = S.SortedCache()
            c[f"m{mid}t{t}"] = S.TR(S.to_dev(fx.weights(f"m{mid}/update{t}"), DEV), 10 + t, rnd - t % 2)
            agg = opt.do(agg, c, total=10 + t, version=rnd)
        new, delta = opt.scale_add_agg_weights_with_delta(mid_w, agg, arr)
        assert new is mid_w
        S.assert_bitwise(f"m{mid}/delta", delta, fx.weights(f"m{mid}/delta"))


@pytest.mark.oracle
@pytest.mark.parametrize("name", S.HIER_FIXTURES)
@pytest.mark.parametrize("update_middle_weights", [True, False])
def test_golden_hier_one_pass(golden, name, update_middle_weights):
    """A reference-generated hierarchy (2 middles x 3 arrivals, bf16; 18 x 2 over f32 / f16 /
    bf16 -- LDS-held store groups) in ONE flame_hier_fedbuff launch per dtype
    (hierarchy_round): middle deltas and the top model bitwise equal the reference's
    (make_golden.py drove flame's own FedBuff + delta_weights)."""
    from flame_amd import engine
    from flame_amd.optimizer.fedbuff import hierarchy_round
    fx = golden(name)
    rnd = fx.meta["round"]
    mids, arr, mver = S.hier_shape(fx.meta)
    top_w0 = fx.weights("top_w0")
    middles = []
    shared = S.to_dev(top_w0, DEV)
    for mid in range(mids):
        opt, agg = make_amd("fedbuff"), None
        for t in range(arr):
            c = S.SortedCache()
            c[f"m{mid}t{t}"] = S.TR(S.to_dev(fx.weights(f"m{mid}/update{t}"), DEV), 10 + t, rnd - t % 2)
            agg = opt.do(agg, c, total=10 + t, version=rnd)
        middles.append((S.to_dev(top_w0, DEV) if update_middle_weights else shared, agg, arr, mver[mid]))
    top = S.to_dev(top_w0, DEV)
    engine.kernel_events = []
    try:
        _, deltas = hierarchy_round(middles, None, version=rnd, top_weights=top, top_goal=mids, with_delta=True,
                                    update_middle_weights=update_middle_weights)
        assert [e[0] for e in engine.kernel_events] == ["flame_hier_fedbuff"] * len({v.dtype for v in top.values()})
    finally:
        engine.kernel_events = None
    for mid in range(mids):
        S.assert_bitwise(f"m{mid}/delta", S.to_cpu(deltas[mid]), fx.weights(f"m{mid}/delta"))
    S.assert_bitwise("top_out", S.to_cpu(top), fx.weights("top_out"))


# ------------------------------------------------------------------ oracle comparisons
def _oracle():
    from oracle import oracle as O
    return O


def _synth_dev(seed, stream, n, sigma, dtype=torch.float32):
    from flame_amd import engine
    t = torch.empty(n, dtype=dtype, device=DEV)
    engine.synth_fill_(t, seed, stream, 0, sigma)
    return t


def test_synth_device_matches_host():
    from flame_amd import synth
    for dt in (torch.float32, torch.bfloat16):
        t = _synth_dev(3, 17, 100_003, 0.01, dt).cpu()
        h = synth.synth_f32(3, 17, 100_003, 0.01)
        if dt == torch.bfloat16:
            assert np.array_equal(t.view(torch.int16).numpy().view(np.uint16), synth.f32_to_bf16_bits(h))
        else:
            assert np.array_equal(t.numpy().view(np.uint32), h.view(np.uint32))


@pytest.mark.oracle
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16, torch.float64,
                                   torch.int64, torch.int32])
@pytest.mark.parametrize("numel", [0, 1, 3, 1023, 1024, 4099, 70_001])
def test_reduce_vs_oracle_dtypes(dtype, numel):
    O = _oracle()
    g = torch.Generator().manual_seed(numel * 7 + 1)
    n = 37
    if dtype.is_floating_point:
        base = torch.randn(numel, generator=g, dtype=torch.float64).to(dtype)
        cl = [(torch.randn(numel, generator=g, dtype=torch.float64) * 1e-2).to(dtype) for _ in range(n)]
    else:
        base = torch.randint(-1000, 1000, (numel,), generator=g, dtype=dtype)
        cl = [torch.randint(-100, 100, (numel,), generator=g, dtype=dtype) for _ in range(n)]
    counts = torch.randint(1, 1000, (n,), generator=g).tolist()
    total = sum(counts)
    exp = base.clone()
    O.reduce_tensor(exp, cl, [c / total for c in counts])
    cache = S.SortedCache()
    for i, (c, k) in enumerate(zip(cl, counts)):
        cache[f"{i:04d}"] = S.TR({"x": c.to(DEV)}, k)
    out = make_amd("fedavg").do({"x": base.to(DEV)}, cache, total=total)
    S.assert_bitwise(f"{dtype}/{numel}", out, {"x": exp})


# (clients, extra small keys, the launch branch the round takes): the low-residency instantiation
# with LDS-held output bursts below 512 clients and without at 512, through the kernel-argument
# metadata (a few keys) and through the device table (more segments x clients than 3.5 KB holds)
LO_CASES = [(64, 0, "flame_agg_reduce_argmeta/lo_burst", "tensors"), (64, 7, "flame_agg_reduce/lo_burst", "tensors"),
            (64, 7, "flame_agg_reduce/lo_burst", "slab"), (512, 1, "flame_agg_reduce/lo", "tensors")]


@pytest.mark.oracle
@pytest.mark.parametrize("case", LO_CASES, ids=[f"n{n}_k{k}_{pl}" for n, k, _, pl in LO_CASES])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
def test_low_residency_reduction_vs_oracle(dtype, case):
    """flame_agg_reduce's 2-workgroups-per-CU instantiations (launches of >= 64 clients over >= 4,096
    chunks; below 512 clients with kLoWGC chunks' outputs held in LDS and stored in bursts; DESIGN.md
    §4) on every element against the oracle: clients as separate tensors (the row layout, so the
    XCD chunk map is on too) or slots of a tiled UpdateSlab (the client tile stride), over one
    4,096-chunk key + small ragged keys (a burst's 8 chunks then straddle keys and tails), every
    float dtype the path instantiates, and the branch each launch took."""
    from flame_amd import _native, engine
    from flame_amd.slab import UpdateSlab
    O = _oracle()
    n, extra, branch, placement = case
    chunk = engine.chunk_elems(engine.dtype_code(dtype))
    shapes = [("w", 4096 * chunk)] + [(f"t{j}", 4_099 + 13 * j) for j in range(extra)]
    g = torch.Generator().manual_seed(11)
    counts = torch.randint(1, 1000, (n,), generator=g).tolist()
    total = sum(counts)
    base = {k: _synth_dev(12, 0 + j, s, 1.0, dtype) for j, (k, s) in enumerate(shapes)}
    cl = [{k: _synth_dev(12, 10 + 2 * i + j, s, 1e-2, dtype) for j, (k, s) in enumerate(shapes)} for i in range(n)]
    exp = {k: v.cpu() for k, v in base.items()}
    rates = [c / total for c in counts]
    for k in exp:
        # the oracle is element-wise: disjoint element ranges reduce in parallel threads (the C
        # call releases the GIL), each in client order
        host = [c[k].cpu() for c in cl]
        parts = [(a, min(a + (1 << 20), exp[k].numel())) for a in range(0, exp[k].numel(), 1 << 20)]
        with concurrent.futures.ThreadPoolExecutor(8) as ex:
            list(ex.map(lambda ab: O.reduce_tensor(exp[k][ab[0]:ab[1]], [h[ab[0]:ab[1]] for h in host], rates),
                        parts))
    if placement == "slab":
        slab = UpdateSlab({k: torch.empty(sz, dtype=dtype) for k, sz in shapes}, capacity=n, device=DEV)
        cl = [slab.put(c) for c in cl]
    cache = S.SortedCache()
    for i in range(n):
        cache[f"{i:04d}"] = S.TR(cl[i], counts[i])
    dt = {torch.float32: "f32", torch.bfloat16: "bf16", torch.float16: "f16"}[dtype]
    before = _native.launch_branch_counts()
    out = make_amd("fedavg").do({k: v.clone() for k, v in base.items()}, cache, total=total)
    torch.cuda.synchronize()
    after = _native.launch_branch_counts()
    hit = {k for k, v in after.items() if v > before.get(k, 0)}
    assert f"{branch}/{dt}" in hit, hit
    S.assert_bitwise(f"low-residency {dtype} n{n}", out, exp)


@pytest.mark.oracle
def test_c2_256x1M_bitwise():
    """Config 2: 256 clients x (1,000,000 + 4,099) fp32, counts U{1..1000}, seed 1."""
    from flame_amd import synth
    O = _oracle()
    n, shapes = 256, [("w", 1_000_000), ("t", 4_099)]
    P = sum(s for _, s in shapes)
    base_flat = _synth_dev(1, 0, P, 1.0)
    clients = [_synth_dev(1, 1 + i, P, 1e-2) for i in range(n)]
    counts = synth.counts(1, n)
    total = int(counts.sum())

    def split(flat):
        out, off = {}, 0
        for k, s in shapes:
            out[k] = flat[off:off + s]
            off += s
        return out
    cache = S.SortedCache()
    for i in range(n):
        cache[f"c{i:04d}"] = S.TR(split(clients[i]), int(counts[i]))
    base = {k: v.clone() for k, v in split(base_flat).items()}
    base_cpu = {k: v.cpu() for k, v in base.items()}
    out = make_amd("fedavg").do(base, cache, total=total)
    for k, _ in shapes:
        exp = base_cpu[k].clone()
        O.reduce_tensor(exp, [split(c)[k].cpu() for c in clients], [int(c) / total for c in counts])
        S.assert_bitwise(f"c2/{k}", {k: out[k]}, {k: exp})


@pytest.mark.oracle
def test_unaligned_and_strided_and_host_base():
    """Views at odd offsets (scalar path), non-contiguous base, CPU-resident base."""
    O = _oracle()
    g = torch.Generator().manual_seed(5)
    n = 9
    big = [torch.randn(5001, generator=g) * 1e-2 for _ in range(n)]
    cl = [b.to(DEV)[1:4998] for b in big]                       # 4-byte misaligned views
    base_full = torch.randn(2, 4997, generator=g)
    counts = list(range(1, n + 1))
    total = sum(counts)
    exp = base_full[1].clone()
    O.reduce_tensor(exp, [b[1:4998].clone() for b in big], [c / total for c in counts])
    # non-contiguous device base (column of a transposed tensor)
    base_dev = base_full.t().contiguous().to(DEV).t()[1]
    assert not base_dev.is_contiguous()
    cache = S.SortedCache()
    for i in range(n):
        cache[f"{i}"] = S.TR({"x": cl[i]}, counts[i])
    base = {"x": base_dev}
    out = make_amd("fedavg").do(base, cache, total=total)
    assert out["x"] is base_dev
    S.assert_bitwise("strided", {"x": base_dev.contiguous()}, {"x": exp})
    # host-resident base and clients (end-to-end path): mutated in place on the host
    cache = S.SortedCache()
    for i in range(n):
        cache[f"{i}"] = S.TR({"x": big[i][1:4998].clone()}, counts[i])
    hb = base_full[1].clone()
    out = make_amd("fedavg").do({"x": hb}, cache, total=total)
    assert out["x"] is hb and hb.device.type == "cpu"
    S.assert_bitwise("host", {"x": hb}, {"x": exp})


def test_fedbuff_errors_and_int_scale_add():
    opt = make_amd("fedbuff")
    c = S.SortedCache()
    c["a"] = S.TR({"w": torch.ones(4, device=DEV)}, 3, 5)
    with pytest.raises(ZeroDivisionError):
        opt.do(None, c, total=3, version=4)          # 1 + 4 - 5 == 0
    c["b"] = S.TR({"w": torch.ones(4, device=DEV)}, 3, 9)
    with pytest.raises(ValueError):
        opt.do(None, c, total=3, version=4)          # sqrt of a negative
    with pytest.raises(RuntimeError):
        opt.scale_add_agg_weights({"n": torch.ones(3, dtype=torch.int64, device=DEV)},
                                  {"n": torch.ones(3, dtype=torch.int64, device=DEV)}, 2)


@pytest.mark.oracle
@pytest.mark.parametrize("sort", ["fedadam", "fedyogi", "fedadagrad"])
def test_fedopt_vs_oracle_random(sort):
    """Four rounds at N=64, P=300,001 fp32 (+ an int64 buffer on the generic path)."""
    O = _oracle()
    g = torch.Generator().manual_seed({"fedadam": 1, "fedyogi": 2, "fedadagrad": 3}[sort])
    P, n, rounds = 300_001, 64, 4
    w0 = torch.randn(P, generator=g)
    data = []
    for r in range(rounds):
        cl = [torch.randn(P, generator=g) * 1e-2 for _ in range(n)]
        counts = torch.randint(1, 1000, (n,), generator=g).tolist()
        data.append((cl, counts))
    amd, ora = make_amd(sort), O.OracleFedOPT(sort)
    wa = {"w": w0.to(DEV), "nbt": torch.tensor(7, dtype=torch.int64, device=DEV)}
    wo = {"w": w0.clone()}
    for r, (cl, counts) in enumerate(data):
        ca, co = S.SortedCache(), S.SortedCache()
        for i in range(n):
            ca[f"{i:03d}"] = S.TR({"w": cl[i].to(DEV), "nbt": torch.tensor(r + 1, device=DEV)}, counts[i])
            co[f"{i:03d}"] = S.TR({"w": cl[i].clone()}, counts[i])
        wa = amd.do({k: v.clone() for k, v in wa.items()}, ca, total=sum(counts))
        wo = ora.do({k: v.clone() for k, v in wo.items()}, co, total=sum(counts))
        if r == 0:
            S.assert_bitwise(f"{sort}/r0", {"w": wa["w"]}, wo)
        else:
            S.assert_close_fedopt(f"{sort}/r{r}/cur", {"w": wa["w"]}, wo)
            S.assert_close_fedopt(f"{sort}/r{r}/m", {"w": amd.m_t["w"]}, {"w": ora.m_t["w"]})
    assert wa["nbt"].dtype == torch.float32  # the reference promotes int buffers in the adaptive step


@pytest.mark.oracle
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_fedbuff_stream_vs_oracle(dtype):
    """FedBuff: 12 single-entry do() calls with staleness 0..3, then scale_add (+delta)."""
    O = _oracle()
    g = torch.Generator().manual_seed(99)
    P = 123_457
    w0 = (torch.randn(P, generator=g)).to(dtype)
    ups = [(torch.randn(P, generator=g) * 1e-2).to(dtype) for _ in range(12)]
    stale = [i % 4 for i in range(12)]
    amd, ora = make_amd("fedbuff"), O.OracleFedBuff()
    aa = ao = None
    for i, u in enumerate(ups):
        ca, co = S.SortedCache(), S.SortedCache()
        ca[f"{i}"] = S.TR({"w": u.to(DEV)}, 5, 10 - stale[i])
        co[f"{i}"] = S.TR({"w": u.clone()}, 5, 10 - stale[i])
        aa = amd.do(aa, ca, total=5, version=10)
        ao = ora.do(ao, co, total=5, version=10)
    S.assert_bitwise(f"fedbuff/{dtype}/agg", S.to_cpu(aa), ao)
    wa = {"w": w0.to(DEV)}
    wo = {"w": w0.clone()}
    new, delta = amd.scale_add_agg_weights_with_delta(wa, aa, 12)
    prev = w0.clone()
    ora.scale_add_agg_weights(wo, ao, 12)
    S.assert_bitwise(f"fedbuff/{dtype}/out", S.to_cpu(new), wo)
    S.assert_bitwise(f"fedbuff/{dtype}/delta", S.to_cpu(delta), {"w": wo["w"] - prev})


def _full_size_columns(P, T, seed):
    """Elements a full-size test checks against the oracle: 65,536 random ones, plus EVERY
    element of whole kernel chunks / slab tiles -- the first two, those at 1/4, 1/2 and 3/4
    of the tensor, and the last two (the last one ragged) -- where tiled addressing
    (client_offset: tile * tile stride + slot) or the chunk -> segment map could go wrong
    without random sampling noticing."""
    n_t = -(-P // T)
    tiles = sorted({0, 1, n_t // 4, n_t // 2, 3 * n_t // 4, n_t - 2, n_t - 1})
    whole = np.concatenate([np.arange(t * T, min((t + 1) * T, P)) for t in tiles])
    rand = np.random.default_rng(seed).choice(P, 65_536, replace=False)
    return np.unique(np.concatenate([whole, rand, [0, P - 1]])), len(whole)


@pytest.mark.oracle
def test_c3_full_size_every_element():
    """Config 3 at full size (1024 x 25M fp32 = 102.4 GB in HBM, the tiled slab the
    headline runs on): EVERY one of the 25M outputs equals the C oracle (fedavg.py:79-104 op
    sequence, cache order), bitwise -- the slab streamed through host memory column chunk by
    column chunk (tests/full_check.py)."""
    import full_check as F
    from flame_amd import synth, engine
    from flame_amd.slab import UpdateSlab
    n, P = 1024, 25_000_000
    free, _ = torch.cuda.mem_get_info()
    if free < (n + 6) * P * 4:
        pytest.skip(f"needs {(n + 6) * P * 4 / 1e9:.1f} GB of HBM, {free / 1e9:.1f} GB free")
    slab = UpdateSlab({"model": torch.empty(P)}, capacity=n, device=DEV)
    tmp = torch.empty(P, device=DEV)
    ws = []
    for i in range(n):
        engine.synth_fill_(tmp, 2, 1 + i, 0, 1e-2)
        ws.append(slab.put({"model": tmp}))
    del tmp
    base = _synth_dev(2, 0, P, 1.0)
    base0 = base.cpu().numpy()
    counts = synth.counts(2, n)
    total = int(counts.sum())
    cache = S.SortedCache()
    for i in range(n):
        cache[f"{i:05d}"] = S.TR(ws[i], int(counts[i]))
    out = make_amd("fedavg").do({"model": base}, cache, total=total)["model"].cpu().numpy()
    rates = [int(c) / total for c in counts]
    bad = checked = 0
    for e0, e1, host in F.columns(slab.storage[torch.float32], n, P):
        acc = base0[e0:e1].copy()
        F.reduce_chunk(host, acc, rates, torch.float32)
        bad += F.mismatches(acc, out[e0:e1])
        checked += e1 - e0
        if e0 == 0:     # the device data is the counter generator's: one column vs the host restatement
            col = np.array([synth.synth_f32(2, 1 + i, np.array([12_345]), 1e-2)[0] for i in range(0, n, 97)])
            assert np.array_equal(col.view(np.uint32), host[::97, 12_345].numpy().view(np.uint32))
    assert checked == P and bad == 0, f"{bad} of {P} elements differ from the oracle"
    del slab, ws, cache
    torch.cuda.empty_cache()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_fedbuff_deferred_equals_per_arrival(dtype):
    """Batched (deferred) FedBuff == one launch per arrival, bitwise, across flush boundaries
    and with intermediate reads of the aggregate."""
    g = torch.Generator().manual_seed(3)
    P = 50_001
    ups = [(torch.randn(P, generator=g) * 1e-2).to(dtype).to(DEV) for _ in range(13)]
    a = make_amd("fedbuff", defer=True, max_pending=5)
    b = make_amd("fedbuff", defer=False)
    aa = ab = None
    for i, u in enumerate(ups):
        ca, cb = S.SortedCache(), S.SortedCache()
        ca["k"] = S.TR({"w": u}, 3, 20 - i % 4)
        cb["k"] = S.TR({"w": u}, 3, 20 - i % 4)
        aa = a.do(aa, ca, total=3, version=20)
        ab = b.do(ab, cb, total=3, version=20)
        if i == 7:  # a read in the middle flushes and must not change the result
            S.assert_bitwise("mid", {"w": aa["w"]}, S.to_cpu(ab))
    S.assert_bitwise("final", S.to_cpu(aa), S.to_cpu(ab))
    wa, wb = {"w": ups[0].clone()}, {"w": ups[0].clone()}
    a.scale_add_agg_weights(wa, aa, 13)
    b.scale_add_agg_weights(wb, ab, 13)
    S.assert_bitwise("scale_add", S.to_cpu(wa), S.to_cpu(wb))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("placement", ["slab", "tensors"])
@pytest.mark.parametrize("with_delta", [False, True])
def test_fedbuff_fused_scale_add(dtype, placement, with_delta):
    """scale_add straight from the queued arrivals (one flame_hier_fedbuff launch, the
    aggregate never materialised) == flush + scale_add, bitwise -- weights, delta, and the
    aggregate itself when it is read afterwards; an already materialised aggregate takes
    the separate path."""
    from flame_amd import engine
    from flame_amd.slab import UpdateSlab
    g = torch.Generator().manual_seed(71)
    shapes = {"w": (3001,), "m": (17, 129), "b": (5,)}
    K, rnd = 11, 9
    ups = [{k: (torch.randn(s, generator=g) * 1e-2).to(dtype) for k, s in shapes.items()} for _ in range(K)]
    w0 = {k: torch.randn(s, generator=g).to(dtype) for k, s in shapes.items()}
    slab = UpdateSlab({k: torch.empty(s, dtype=dtype) for k, s in shapes.items()}, capacity=2 * K, device=DEV) \
        if placement == "slab" else None
    res = {}
    for fuse in (True, False):
        opt, agg = make_amd("fedbuff", fuse_scale_add=fuse), None
        for i, u in enumerate(ups):
            w = {k: v.to(DEV) for k, v in u.items()}
            cache = S.SortedCache()
            cache["a"] = S.TR(slab.put(w) if slab is not None else w, 1, rnd - i % 4)
            agg = opt.do(agg, cache, total=1, version=rnd)
        base = {k: v.to(DEV) for k, v in w0.items()}
        launches = []
        engine._recorders.append(launches)
        try:
            if with_delta:
                _, delta = opt.scale_add_agg_weights_with_delta(base, agg, K)
            else:
                opt.scale_add_agg_weights(base, agg, K)
                delta = None
        finally:
            engine._recorders.remove(launches)
        names = [e[0] for e in launches]
        if fuse:
            assert names == ["flame_hier_fedbuff"], names    # one launch per dtype (3 keys, one dtype)
        else:
            assert "flame_hier_fedbuff" not in names, names
        res[fuse] = (S.to_cpu(base), S.to_cpu(delta) if delta is not None else None, S.to_cpu(dict(agg)))
        del agg
    S.assert_bitwise("fused base", res[True][0], res[False][0])
    if with_delta:
        S.assert_bitwise("fused delta", res[True][1], res[False][1])
    S.assert_bitwise("aggregate read afterwards", res[True][2], res[False][2])


@pytest.mark.oracle
def test_zero_copy_pinned_host_clients():
    """Pinned host updates are streamed by the kernel directly (no staging copy): bitwise."""
    O = _oracle()
    from flame_amd import engine
    assert engine.ZERO_COPY_PINNED
    g = torch.Generator().manual_seed(11)
    P, n = 300_007, 23
    cl = [(torch.randn(P, generator=g) * 1e-2).pin_memory() for _ in range(n)]
    base = torch.randn(P, generator=g)
    counts = list(range(5, 5 + n))
    exp = base.clone()
    O.reduce_tensor(exp, cl, [c / sum(counts) for c in counts])
    cache = S.SortedCache()
    for i in range(n):
        cache[f"{i:03d}"] = S.TR({"x": cl[i]}, counts[i])
    out = make_amd("fedavg").do({"x": base.to(DEV)}, cache, total=sum(counts))
    S.assert_bitwise("zerocopy", S.to_cpu(out), {"x": exp})


@pytest.mark.oracle
@pytest.mark.parametrize("where", ["bytes", "pinned", "cache_hbm", "cache_host", "cache_slab"])
def test_ingest_wire_payloads_to_fedavg(where):
    """Channel payloads (cloudpickle, channel.py:203-218) -> ingest.decode (zero-copy) ->
    FedAvg on the GPU == oracle on the original tensors, bitwise."""
    import cloudpickle
    from flame_amd import ingest
    O = _oracle()
    g = torch.Generator().manual_seed(21)
    n = 12
    ws = [{"w": torch.randn(4097, 3, generator=g) * 1e-2, "b": (torch.randn(65, generator=g) * 1e-2).bfloat16(),
           "nbt": torch.tensor(i, dtype=torch.int64)} for i in range(n)]
    base = {"w": torch.randn(4097, 3, generator=g), "b": torch.randn(65, generator=g).bfloat16(),
            "nbt": torch.tensor(100, dtype=torch.int64)}
    counts = [10 + 7 * i for i in range(n)]
    total = sum(counts)
    keep = []
    cache = ingest.DeviceUpdateCache(placement=where.split("_")[1], capacity=16) \
        if where.startswith("cache") else S.SortedCache()
    for i in range(n):
        b = cloudpickle.dumps({"weights": ws[i], "dataset_size": counts[i]})
        if where == "pinned":
            pb = torch.empty(len(b), dtype=torch.uint8, pin_memory=True)
            pb.numpy()[:] = memoryview(b)
            b = pb.numpy()
        keep.append(b)
        msg = ingest.decode(b)
        if where == "pinned":
            assert all(t.is_pinned() for t in msg["weights"].values() if t.numel())
        cache[f"{i:03d}"] = S.TR(msg["weights"], msg["dataset_size"])
    out = make_amd("fedavg").do({k: v.to(DEV) for k, v in base.items()}, cache, total=total)
    for k in base:
        exp = base[k].clone()
        O.reduce_tensor(exp, [w[k] for w in ws], [c / total for c in counts])
        S.assert_bitwise(f"{where}/{k}", {k: out[k]}, {k: exp})


def _slab_model(g):
    from flame_amd import engine
    T = engine.chunk_elems(0)
    return {"big": torch.randn(3 * T + 17, generator=g), "tiny": torch.randn(5, generator=g),
            "exact": torch.randn(T, generator=g), "bf": torch.randn(2 * 2048 + 3, generator=g).bfloat16(),
            "mat": torch.randn(33, 65, generator=g), "nbt": torch.tensor(7, dtype=torch.int64)}


@pytest.mark.oracle
def test_slab_tiled_fedavg_bitwise_and_slot_reuse():
    """Updates in the tiled UpdateSlab (client_tile_stride path) == oracle, bitwise; slots
    released after the round are reused by the next one."""
    from flame_amd import engine
    from flame_amd.slab import UpdateSlab
    O = _oracle()
    g = torch.Generator().manual_seed(8)
    tmpl = _slab_model(g)
    slab = UpdateSlab(tmpl, capacity=40, device=DEV)
    base = {k: v.clone() for k, v in tmpl.items()}
    for rnd in range(2):
        n = 37
        ws = [{k: (torch.randn(v.shape, generator=g) * 1e-2).to(v.dtype) if v.is_floating_point()
               else torch.tensor(i, dtype=v.dtype) for k, v in tmpl.items()} for i in range(n)]
        counts = [3 + 5 * i for i in range(n)]
        cache = S.SortedCache()
        for i in range(n):
            sw = slab.put({k: v.to(DEV) for k, v in ws[i].items()})
            assert engine.tiled_stride(sw["big"], tmpl["big"].numel()) == 40 * engine.chunk_elems(0) * 4
            cache[f"{i:03d}"] = S.TR(sw, counts[i])
        del sw
        dev_base = {k: v.to(DEV) for k, v in base.items()}
        out = make_amd("fedavg").do(dev_base, cache, total=sum(counts))
        for k in base:
            exp = base[k].clone()
            O.reduce_tensor(exp, [w[k] for w in ws], [c / sum(counts) for c in counts])
            S.assert_bitwise(f"slab r{rnd}/{k}", {k: out[k]}, {k: exp})
            base[k] = exp
        import gc
        gc.collect()
        assert len(slab._free) == 40, "slots must return after the round"


@pytest.mark.oracle
def test_slab_fedopt_and_fedbuff_tiled():
    from flame_amd.slab import UpdateSlab
    O = _oracle()
    g = torch.Generator().manual_seed(9)
    P = 100_003
    slab = UpdateSlab({"w": torch.zeros(P)}, capacity=16, device=DEV)
    w0 = torch.randn(P, generator=g)
    amd, ora = make_amd("fedadam"), O.OracleFedOPT("fedadam")
    wa, wo = {"w": w0.to(DEV)}, {"w": w0.clone()}
    for r in range(3):
        ups = [torch.randn(P, generator=g) * 1e-2 for _ in range(12)]
        counts = [10 + i for i in range(12)]
        ca, co = S.SortedCache(), S.SortedCache()
        for i in range(12):
            ca[f"{i:02d}"] = S.TR(slab.put({"w": ups[i].to(DEV)}), counts[i])
            co[f"{i:02d}"] = S.TR({"w": ups[i]}, counts[i])
        wa = amd.do({"w": wa["w"].clone()}, ca, total=sum(counts))
        wo = ora.do({"w": wo["w"].clone()}, co, total=sum(counts))
        if r == 0:
            S.assert_bitwise("slab fedadam r0", S.to_cpu(wa), wo)
        else:
            S.assert_close_fedopt(f"slab fedadam r{r}", S.to_cpu(wa), wo)
    # FedBuff: deferred arrivals from slab slots
    fb, ob = make_amd("fedbuff"), O.OracleFedBuff()
    aa = ao = None
    for i in range(10):
        u = torch.randn(P, generator=g) * 1e-2
        ca, co = S.SortedCache(), S.SortedCache()
        ca["x"] = S.TR(slab.put({"w": u.to(DEV)}), 1, 5 - i % 3)
        co["x"] = S.TR({"w": u}, 1, 5 - i % 3)
        aa = fb.do(aa, ca, total=1, version=5)
        ao = ob.do(ao, co, total=1, version=5)
    S.assert_bitwise("slab fedbuff", S.to_cpu(aa), ao)


@pytest.mark.oracle
def test_registered_shared_memory_payloads_zero_copy():
    """Payloads in a registered mmap (stand-in for the LIFL shm segment) are decoded in
    place and read by the kernel over PCIe: no host copy anywhere, result bitwise."""
    import mmap
    import cloudpickle
    from flame_amd import ingest
    O = _oracle()
    g = torch.Generator().manual_seed(31)
    n, P = 6, 50_021
    ws = [{"w": torch.randn(P, generator=g) * 1e-2} for _ in range(n)]
    blobs = [cloudpickle.dumps({"weights": w, "dataset_size": 10 + i}) for i, w in enumerate(ws)]
    size = sum(len(b) for b in blobs)
    mm = mmap.mmap(-1, (size + 4095) // 4096 * 4096)
    offs, o = [], 0
    for b in blobs:
        mm[o:o + len(b)] = b
        offs.append(o)
        o += len(b)
    with ingest.RegisteredBuffer(mm) as reg:
        mv = memoryview(mm)
        cache = S.SortedCache()
        for i, (b, off) in enumerate(zip(blobs, offs)):
            msg = ingest.decode(mv[off:off + len(b)])
            assert msg["weights"]["w"].is_pinned()
            cache[f"{i}"] = S.TR(msg["weights"], msg["dataset_size"])
        base = torch.randn(P, generator=g)
        out = make_amd("fedavg").do({"w": base.to(DEV)}, cache, total=sum(10 + i for i in range(n)))
        torch.cuda.synchronize()
        exp = base.clone()
        O.reduce_tensor(exp, [w["w"] for w in ws], [(10 + i) / sum(10 + j for j in range(n)) for i in range(n)])
        S.assert_bitwise("registered", S.to_cpu(out), {"w": exp})
        del cache, msg


@pytest.mark.oracle
@pytest.mark.parametrize("sort", ["fedadam", "fedyogi", "fedadagrad"])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_fedopt_fused_reduced_precision_vs_reference_ops(sort, dtype):
    """bf16 / fp16 FedOPT keys take the fused kernel; compare with the reference's own torch-CPU
    op sequence (oracle._adapt_torch) over 3 rounds: the reduction is bitwise, and so is the
    adaptive step -- current, m and v.  (torch-CPU's fp32 sqrt is not always correctly rounded,
    but an fp32 root within an ulp rounds to the same bf16 / fp16 value: tools/fp_probe.py checks
    that exhaustively for the hardware root)"""
    O = _oracle()
    g = torch.Generator().manual_seed(17)
    P, n = 20_011, 8
    w0 = torch.randn(P, generator=g).to(dtype)
    amd, ora = make_amd(sort), O.OracleFedOPT(sort)
    wa, wo = {"w": w0.to(DEV)}, {"w": w0.clone()}
    ulp = 2.0 ** -7 if dtype == torch.bfloat16 else 2.0 ** -10
    for r in range(3):
        cl = [(torch.randn(P, generator=g) * 1e-2).to(dtype) for _ in range(n)]
        counts = [5 + 3 * i for i in range(n)]
        ca, co = S.SortedCache(), S.SortedCache()
        for i in range(n):
            ca[f"{i}"] = S.TR({"w": cl[i].to(DEV)}, counts[i])
            co[f"{i}"] = S.TR({"w": cl[i].clone()}, counts[i])
        wa = amd.do({"w": wa["w"].clone()}, ca, total=sum(counts))
        wo = ora.do({"w": wo["w"].clone()}, co, total=sum(counts))
        S.assert_bitwise(f"{sort}/{dtype}/r{r}/avg", S.to_cpu(amd.agg_weights), ora.agg_weights)
        got, exp = wa["w"].cpu().double(), wo["w"].double()
        assert got.dtype == exp.dtype and wa["w"].dtype == dtype
        tiny = 2.0 ** -24 if dtype == torch.float16 else 1e-30   # one fp16 subnormal ulp
        bad = ((got - exp).abs() > exp.abs() * ulp + tiny).nonzero().flatten()
        assert bad.numel() == 0, f"{sort}/{dtype}/r{r}: {bad.numel()} off, {got[bad[:4]]} vs {exp[bad[:4]]}"
        S.assert_bitwise(f"{sort}/{dtype}/r{r}/current", S.to_cpu(wa), wo)
        if r >= 1:
            assert amd.m_t["w"].dtype == dtype
            S.assert_bitwise(f"{sort}/{dtype}/r{r}/m", S.to_cpu(amd.m_t), ora.m_t)
            S.assert_bitwise(f"{sort}/{dtype}/r{r}/v", S.to_cpu(amd.v_t), ora.v_t)
        wo = {"w": wa["w"].cpu().clone()}   # continue both from the same state
        if ora.current_weights is not None:
            ora.current_weights = {"w": wo["w"].clone()}
        if amd.m_t is not None and ora.m_t is not None:
            ora.m_t = {"w": amd.m_t["w"].cpu().clone()}
            ora.v_t = {"w": amd.v_t["w"].cpu().clone()}


def _dyn_model(g, P):
    return {"w": torch.randn(P, generator=g), "m": torch.randn(31, 129, generator=g),
            "bf": torch.randn(4099, generator=g).bfloat16(), "h": torch.randn(777, generator=g).half(),
            "d": torch.randn(2051, generator=g).double(), "nbt": torch.tensor(3, dtype=torch.int64)}


def _dyn_update(g, tmpl, i, scale=1e-2):
    return {k: (torch.randn(v.shape, generator=g) * scale).to(v.dtype) if v.is_floating_point()
            else torch.tensor(i, dtype=v.dtype) for k, v in tmpl.items()}


@pytest.mark.oracle
@pytest.mark.parametrize("placement,order,history", [
    ("hbm", "sorted", "rows"), ("slab", "sorted", "rows"), ("hbm", "shuffled", "rows"), ("slab", "shuffled", "rows"),
    ("hbm", "sorted", "pingpong"), ("slab", "shuffled", "pingpong"), ("slab", "shuffled", "pingpong_rows")])
def test_feddyn_vs_oracle_partial_participation(placement, order, history):
    """FedDyn drop-in == oracle bitwise over 4 rounds with ends dropping out, returning and
    one untracked end; updates device-resident or tiled UpdateSlab views (history copies
    are untiled).  ~1M params x 24 ends.  ``sorted`` active_ends = the cache order (one
    merged flame_feddyn_round program); ``shuffled`` = the channel's join order differs, so
    the mean re-reads the updated histories in a second phase.  ``pingpong``: histories in
    two tiled stores, each round writing the other one (the end that leaves frees its slot)."""
    from flame_amd.slab import UpdateSlab
    O = _oracle()
    g = torch.Generator().manual_seed(23)
    tmpl = _dyn_model(g, 1_000_003)
    all_ends = [f"e{i:02d}" for i in range(24)]
    if order == "shuffled":
        all_ends = [all_ends[i] for i in np.random.default_rng(7).permutation(24)]
    rounds = [all_ends[:16], all_ends[4:], all_ends[::3] + ["zz"], all_ends[1::2]]
    slab = UpdateSlab(tmpl, capacity=48, device=DEV) if placement == "slab" else None
    from flame_amd import engine
    launches = []
    engine._recorders.append(launches)
    amd, ora = make_amd("feddyn", alpha=0.01, history=history), O.OracleFedDyn(alpha=0.01)
    ca_w, co_w = {k: v.to(DEV) for k, v in tmpl.items()}, {k: v.clone() for k, v in tmpl.items()}
    for r, ends in enumerate(rounds):
        amd.save_state(S._PRE, active_ends=all_ends)
        ora.save_state(S._PRE, active_ends=all_ends)
        ws = [_dyn_update(g, tmpl, 10 * r + i) for i in range(len(ends))]
        counts = [7 + i for i in range(len(ends))]
        ca, co = S.SortedCache(), S.SortedCache()
        for e, w, c in zip(ends, ws, counts):
            dw = {k: v.to(DEV) for k, v in w.items()}
            ca[e] = S.TR(slab.put(dw) if slab is not None else dw, c)
            co[e] = S.TR({k: v.clone() for k, v in w.items()}, c)
        a = amd.do({k: v.clone() for k, v in ca_w.items()}, ca, total=sum(counts))
        o = ora.do({k: v.clone() for k, v in co_w.items()}, co, total=sum(counts))
        S.assert_bitwise(f"feddyn/{placement}/r{r}/avg", S.to_cpu(a), o)
        S.assert_bitwise(f"feddyn/{placement}/r{r}/cld", S.to_cpu(amd.cld_model), ora.cld_model)
        ca_w, co_w = amd.cld_model, ora.cld_model
        del ca, co
    engine._recorders.remove(launches)
    # float keys (f32, bf16, f16, f64 groups) run as one flame_feddyn_round per dtype each round
    assert sum(1 for ev in launches if ev[0] == "flame_feddyn_round") == 4 * len(rounds)
    assert list(amd.local_param_dict) == list(ora.local_param_dict)
    for e, h in ora.local_param_dict.items():
        if h is not None:
            S.assert_bitwise(f"feddyn/{placement}/hist/{e}", S.to_cpu(amd.local_param_dict[e]), h)


@pytest.mark.oracle
@pytest.mark.parametrize("history", ["pingpong", "pingpong_rows"])
def test_feddyn_pingpong_key_leaves_and_returns(history):
    """under history="pingpong" a key whose arrival comes in another dtype takes the
    reference path for that round; the arriving ends' updated histories must land back in the
    stores (a new end included), so the next fused round reads them -- and a history torch
    promoted to a wider dtype (f32 + f64 -> f64) keeps the key off the fused path while any
    end holds it.  5 rounds vs the oracle, bitwise: average, cld_model, every history."""
    O = _oracle()
    g = torch.Generator().manual_seed(61)
    tmpl = _dyn_model(g, 300_007)
    ends0 = [f"e{i}" for i in range(6)]
    rounds = [
        (ends0, {}),                                              # all fused
        (ends0[:4] + ["n1"], {"e1": ("w", torch.bfloat16)}),      # w -> reference path; n1 new
        (["e0", "e1", "n1", "e5"], {}),                           # w fused again: reads the stores
        (["e2", "e3", "n2"], {"e2": ("w", torch.float64)}),       # e2's history of w becomes f64
        (ends0 + ["n1", "n2"], {}),                               # w stays on the reference path
    ]
    amd = make_amd("feddyn", alpha=0.01, history=history)
    ora = O.OracleFedDyn(alpha=0.01)
    wa, wo = {k: v.to(DEV) for k, v in tmpl.items()}, {k: v.clone() for k, v in tmpl.items()}
    every = ends0 + ["n1", "n2"]
    for r, (ends, odd) in enumerate(rounds):
        amd.save_state(S._PRE, active_ends=every)
        ora.save_state(S._PRE, active_ends=every)
        ca, co = S.SortedCache(), S.SortedCache()
        for i, e in enumerate(ends):
            u = _dyn_update(g, tmpl, 10 * r + i)
            if e in odd:
                k, dt = odd[e]
                u[k] = u[k].to(dt)
            ca[e] = S.TR({k: v.to(DEV) for k, v in u.items()}, 5 + i)
            co[e] = S.TR({k: v.clone() for k, v in u.items()}, 5 + i)
        total = sum(5 + i for i in range(len(ends)))
        a = amd.do({k: v.clone() for k, v in wa.items()}, ca, total=total)
        o = ora.do({k: v.clone() for k, v in wo.items()}, co, total=total)
        S.assert_bitwise(f"pp/{history}/r{r}/avg", S.to_cpu(a), o)
        S.assert_bitwise(f"pp/{history}/r{r}/cld", S.to_cpu(amd.cld_model), ora.cld_model)
        for e, h in ora.local_param_dict.items():
            if h is not None:
                got = {k: amd.local_param_dict[e][k] for k in h}
                S.assert_bitwise(f"pp/{history}/r{r}/hist/{e}", S.to_cpu(got), h)
        wa, wo = amd.cld_model, ora.cld_model


@pytest.mark.oracle
def test_scaffold_vs_oracle_rounds():
    """SCAFFOLD drop-in == oracle bitwise: c_glob (HBM-resident, updated in place) and the
    model over 3 rounds, including an int buffer whose control variate arrives as fp32, and
    the None results (empty cache; control/model cache length mismatch) leave state alone."""
    O = _oracle()
    g = torch.Generator().manual_seed(29)
    tmpl = _dyn_model(g, 500_009)
    ends = [f"t{i:02d}" for i in range(20)]
    sizes = {e: 100 + 37 * i for i, e in enumerate(ends)}
    amd, ora = make_amd("scaffold", k=3), O.OracleScaffold(k=3)
    for o in (amd, ora):
        o.save_state(S._PRE, dataset_sizes=sizes)
    wa, wo = {k: v.to(DEV) for k, v in tmpl.items()}, {k: v.clone() for k, v in tmpl.items()}
    for r, rends in enumerate([ends[:12], ends[5:], ends[::2]]):
        amd.save_state(S._PRE, glob_weights=wa)
        ora.save_state(S._PRE, glob_weights=wo)
        ws = [_dyn_update(g, tmpl, r + i) for i in range(len(rends))]
        cs = [_dyn_update(g, tmpl, 0, 1e-3) for _ in rends]
        for i, c in enumerate(cs):
            c["nbt"] = torch.tensor(9.25 * (i + 1) + r)
        caches = {}
        for side in ("a", "o"):
            mv = (lambda t: t.to(DEV)) if side == "a" else (lambda t: t.clone())
            cache, cc = S.SortedCache(), S.SortedCache()
            for e, w, c in zip(rends, ws, cs):
                cache[e] = S.TR({k: mv(v) for k, v in w.items()}, sizes[e])
                cc[e] = S.TR({k: mv(v) for k, v in c.items()})
            caches[side] = (cache, cc)
        total = sum(sizes[e] for e in rends)
        if r == 1:   # mismatched control cache -> None before anything is consumed
            extra = S.SortedCache()
            assert amd.do(wa, caches["a"][0], total=total, control_cache=extra) is None
            assert len(caches["a"][0]) == len(rends)
            assert amd.do(wa, S.SortedCache(), total=total, control_cache=caches["a"][1]) is None
        wa = amd.do({k: v.clone() for k, v in wa.items()}, caches["a"][0], total=total,
                    control_cache=caches["a"][1])
        wo = ora.do({k: v.clone() for k, v in wo.items()}, caches["o"][0], total=total,
                    control_cache=caches["o"][1])
        S.assert_bitwise(f"scaffold/r{r}/out", S.to_cpu(wa), wo)
        S.assert_bitwise(f"scaffold/r{r}/c_glob", S.to_cpu(amd.c_glob), ora.c_glob)
        assert all(t.is_cuda for t in amd.c_glob.values())


@pytest.mark.oracle
def test_f16_product_keeps_two_roundings():
    """torch computes an fp16 `v * rate` as fp32 product -> fp16 (two roundings).  Inputs are
    chosen where one rounding of the exact product differs (what v_fma_mixlo_f16 would give),
    including fp16 subnormal results; the kernel must match torch on every one."""
    O = _oracle()
    g = torch.Generator().manual_seed(31)
    v = (torch.randn(4_000_000, generator=g) * torch.tensor([1.0, 1e-3, 3e-5]).repeat(1_333_334)[:4_000_000]).half()
    rate = 0.3713
    r32 = torch.tensor(rate, dtype=torch.float32).double()
    # exact product (float64 holds it), rounded once -- numpy converts float64 -> fp16 directly
    once = torch.from_numpy((v.double().numpy() * r32.item()).astype(np.float16))
    twice = (v.float() * torch.tensor(rate, dtype=torch.float32)).half()
    sel = (once.view(torch.int16) != twice.view(torch.int16)).nonzero().flatten()
    assert sel.numel() > 100, "need double-rounding witnesses"
    vs = v[sel].contiguous()
    from flame_amd import engine
    out = torch.zeros(vs.numel(), dtype=torch.half, device=DEV)
    engine.reduce_([out], [out], [[vs.to(DEV)]], [rate])
    exp = torch.zeros(vs.numel(), dtype=torch.half)
    O.reduce_tensor(exp, [vs], [rate])
    S.assert_bitwise("f16 product", {"x": out}, {"x": exp})
    S.assert_bitwise("f16 product torch", {"x": out}, {"x": torch.zeros_like(vs) + vs * rate})


@pytest.mark.oracle
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_middle_group_flush_and_scale_add_many(dtype):
    """Co-located middle aggregators: flush_aggregates + scale_add_many (FLAME_AGG_SEG_RATES,
    one launch per group) == each middle's own FedBuff path, bitwise, and == the oracle.
    Middles differ in staleness and arrival count; round 2 accumulates into round 1's
    aggregate (non-None start)."""
    from flame_amd.optimizer.fedbuff import flush_aggregates, scale_add_many
    O = _oracle()
    g = torch.Generator().manual_seed(37)
    shapes = {"w": (3001,), "m": (17, 129)}
    M, rnd = 6, 9
    arrivals = [5, 5, 5, 3, 5, 3]
    base0 = [{k: torch.randn(s, generator=g).to(dtype) for k, s in shapes.items()} for _ in range(M)]
    ups = [[{k: (torch.randn(s, generator=g) * 1e-2).to(dtype) for k, s in shapes.items()}
            for _ in range(arrivals[m])] for m in range(M)]
    vers = [[rnd - ((m + t) % 4) for t in range(arrivals[m])] for m in range(M)]

    def feed(opt, agg, m, t):
        cache = S.SortedCache()
        cache["a"] = S.TR({k: v.to(DEV) for k, v in ups[m][t].items()}, 1, vers[m][t])
        return opt.do(agg, cache, total=1, version=rnd)

    # group path: two rounds of arrivals into the same aggregates, then one group scale_add
    gopts, gaggs = [make_amd("fedbuff") for _ in range(M)], [None] * M
    iopts, iaggs = [make_amd("fedbuff") for _ in range(M)], [None] * M
    oopts, oaggs = [O.OracleFedBuff() for _ in range(M)], [None] * M
    half = [a // 2 + 1 for a in arrivals]
    for lo, hi in ((0, None), (None, None)):
        for m in range(M):
            rng_t = range(0, half[m]) if lo == 0 else range(half[m], arrivals[m])
            for t in rng_t:
                gaggs[m] = feed(gopts[m], gaggs[m], m, t)
                iaggs[m] = feed(iopts[m], iaggs[m], m, t)
                cache = S.SortedCache()
                cache["a"] = S.TR({k: v.clone() for k, v in ups[m][t].items()}, 1, vers[m][t])
                oaggs[m] = oopts[m].do(oaggs[m], cache, total=1, version=rnd)
        flush_aggregates(gaggs)
        assert all(not a._pending for a in gaggs)
    gb = [{k: v.to(DEV) for k, v in b.items()} for b in base0]
    ib = [{k: v.to(DEV) for k, v in b.items()} for b in base0]
    res = scale_add_many(list(zip(gb, gaggs)), 4, with_delta=True)
    for m in range(M):
        S.assert_bitwise(f"group agg m{m}", S.to_cpu(gaggs[m].materialize()), S.to_cpu(iaggs[m].materialize()))
        S.assert_bitwise(f"oracle agg m{m}", S.to_cpu(gaggs[m].materialize()), oaggs[m])
        _, idelta = iopts[m].scale_add_agg_weights_with_delta(ib[m], iaggs[m], 4)
        assert res[m][0] is gb[m]
        S.assert_bitwise(f"group base m{m}", S.to_cpu(gb[m]), S.to_cpu(ib[m]))
        S.assert_bitwise(f"group delta m{m}", S.to_cpu(res[m][1]), S.to_cpu(idelta))
        ob = {k: v.clone() for k, v in base0[m].items()}
        O.OracleFedBuff().scale_add_agg_weights(ob, oaggs[m], 4)
        S.assert_bitwise(f"oracle base m{m}", S.to_cpu(gb[m]), ob)


@pytest.mark.oracle
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("placement", ["slab", "tensors", "mixed"])
@pytest.mark.parametrize("top_start", ["none", "existing"])
@pytest.mark.parametrize("M", [5, 21])
@pytest.mark.parametrize("path", ["argmeta", "table"])
def test_hierarchy_round_one_pass(dtype, placement, top_start, M, path, monkeypatch):
    """flame_hier_fedbuff (the co-located middles + top in ONE launch) == the separate
    launches (scale_add_agg_weights_with_delta per middle, top FedBuff.do per delta,
    top scale_add) == the oracle's op sequence, bitwise: top aggregate, top weights,
    middle weights and deltas.  M = 5 takes the register store groups, M = 21 the LDS-held
    groups of 16 (>= kHLdsMinMids) with a partial last group; both through the kernel-argument
    launch and the device-table one (engine.ARGMETA off)."""
    from flame_amd import engine
    from flame_amd.optimizer.fedbuff import hierarchy_round, _compose_hierarchy
    from flame_amd.slab import UpdateSlab
    O = _oracle()
    if path == "table":
        monkeypatch.setattr(engine, "ARGMETA", False)
    g = torch.Generator().manual_seed(41)
    shapes = {"w": (3001,), "m": (17, 129), "b": (5,)}
    C, rnd = 4, 12
    ups = [[{k: (torch.randn(s, generator=g) * 1e-2).to(dtype) for k, s in shapes.items()} for _ in range(C)]
           for _ in range(M)]
    vers = [[rnd - ((m + t) % 4) for t in range(C)] for m in range(M)]
    mid0 = [{k: torch.randn(s, generator=g).to(dtype) for k, s in shapes.items()} for _ in range(M)]
    top_w0 = {k: torch.randn(s, generator=g).to(dtype) for k, s in shapes.items()}
    top_prev = {k: (torch.randn(s, generator=g) * 1e-3).to(dtype) for k, s in shapes.items()}
    mid_ver = [rnd - (m % 3) for m in range(M)]
    goals = [[C, C + 1, C, 3, C][m % 5] for m in range(M)]
    slab = UpdateSlab({k: torch.empty(s, dtype=dtype) for k, s in shapes.items()}, capacity=M * C, device=DEV) \
        if placement != "tensors" else None

    def arrivals():
        opts, aggs = [make_amd("fedbuff") for _ in range(M)], [None] * M
        for m in range(M):
            for t in range(C):
                w = {k: v.to(DEV) for k, v in ups[m][t].items()}
                cache = S.SortedCache()
                # "mixed": a middle's arrivals alternate between slab slots and plain tensors
                in_slab = slab is not None and (placement == "slab" or (m + t) % 2 == 0)
                cache["a"] = S.TR(slab.put(w) if in_slab else w, 1, vers[m][t])
                aggs[m] = opts[m].do(aggs[m], cache, total=1, version=rnd)
        return aggs

    def run(fn):
        mids = [{k: v.to(DEV) for k, v in b.items()} for b in mid0]
        tw = {k: v.to(DEV) for k, v in top_w0.items()}
        tprev = {k: v.to(DEV) for k, v in top_prev.items()} if top_start == "existing" else None
        mids_in = [(mids[m], a, goals[m], mid_ver[m]) for m, a in enumerate(arrivals())]
        agg, deltas = fn(mids_in, tprev, rnd, tw, 7, True)
        return S.to_cpu(dict(agg)), [S.to_cpu(d) for d in deltas], [S.to_cpu(x) for x in mids], S.to_cpu(tw)

    fused = run(lambda mi, ta, v, tw, tg, wd: hierarchy_round(mi, ta, version=v, top_weights=tw, top_goal=tg,
                                                               with_delta=wd))
    sep = run(_compose_hierarchy)
    for lbl, a, b in zip(("top agg", "deltas", "mids", "top w"), fused, sep):
        if isinstance(a, list):
            for m, (x, y) in enumerate(zip(a, b)):
                S.assert_bitwise(f"{lbl} m{m}", x, y)
        else:
            S.assert_bitwise(lbl, a, b)
    # oracle: the reference's op sequence on CPU
    top_o, top_agg_o = O.OracleFedBuff(), ({k: v.clone() for k, v in top_prev.items()}
                                             if top_start == "existing" else None)
    for m in range(M):
        mo, agg_o = O.OracleFedBuff(), None
        for t in range(C):
            cache = S.SortedCache()
            cache["a"] = S.TR({k: v.clone() for k, v in ups[m][t].items()}, 1, vers[m][t])
            agg_o = mo.do(agg_o, cache, total=1, version=rnd)
        w = {k: v.clone() for k, v in mid0[m].items()}
        d = {k: O.scale_add_tensor(w[k], agg_o[k], goals[m], want_delta=True) for k in w}
        S.assert_bitwise(f"oracle mid m{m}", fused[2][m], w)
        S.assert_bitwise(f"oracle delta m{m}", fused[1][m], d)
        cache = S.SortedCache()
        cache["d"] = S.TR(d, 1, mid_ver[m])
        top_agg_o = top_o.do(top_agg_o, cache, total=1, version=rnd)
    S.assert_bitwise("oracle top agg", fused[0], top_agg_o)
    tw = {k: v.clone() for k, v in top_w0.items()}
    top_o.scale_add_agg_weights(tw, top_agg_o, 7)
    S.assert_bitwise("oracle top w", fused[3], tw)


@pytest.mark.oracle
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("placement", ["slab", "tensors"])
@pytest.mark.parametrize("start", ["none", "existing"])
@pytest.mark.parametrize("defer", [True, False])
def test_fedbuff_do_arrivals_equals_per_do(dtype, placement, start, defer):
    """FedBuff.do_arrivals (a middle's round of arrivals in one call) == do() per arrival (the
    async roles, asyncfl/middle_aggregator.py:190-203) == the oracle, bitwise: the aggregate
    read back, and the fused scale_add + delta applied from the queued arrivals."""
    from flame_amd.slab import UpdateSlab
    O = _oracle()
    g = torch.Generator().manual_seed(77)
    shapes = {"w": (4099,), "m": (33, 65), "b": (3,)}
    n, rnd = 13, 20
    ups = [{k: (torch.randn(sh, generator=g) * 1e-2).to(dtype) for k, sh in shapes.items()} for _ in range(n)]
    vers = [rnd - (i * 3) % 5 for i in range(n)]
    base0 = {k: torch.randn(sh, generator=g).to(dtype) for k, sh in shapes.items()}
    prev = {k: (torch.randn(sh, generator=g) * 1e-3).to(dtype) for k, sh in shapes.items()}
    slab = UpdateSlab({k: torch.empty(sh, dtype=dtype) for k, sh in shapes.items()}, capacity=2 * n, device=DEV) \
        if placement == "slab" else None

    def dev(w):
        w = {k: v.to(DEV) for k, v in w.items()}
        return slab.put(w) if slab is not None else w

    def start_agg():
        return {k: v.to(DEV) for k, v in prev.items()} if start == "existing" else None

    per, agg_p = make_amd("fedbuff"), start_agg()
    for i in range(n):
        c = S.SortedCache()
        c[f"{i}"] = S.TR(dev(ups[i]), 1, vers[i])
        agg_p = per.do(agg_p, c, total=1, version=rnd)
    bat = make_amd("fedbuff", defer=defer)       # defer=False: one launch, a plain dict
    agg_b = bat.do_arrivals(start_agg(), [S.TR(dev(ups[i]), 1, vers[i]) for i in range(n)], version=rnd)
    ora, agg_o = O.OracleFedBuff(), ({k: v.clone() for k, v in prev.items()} if start == "existing" else None)
    for i in range(n):
        c = S.SortedCache()
        c[f"{i}"] = S.TR({k: v.clone() for k, v in ups[i].items()}, 1, vers[i])
        agg_o = ora.do(agg_o, c, total=1, version=rnd)
    # the fused scale_add + delta straight from the queued arrivals (before any read)
    wb = {k: v.to(DEV) for k, v in base0.items()}
    _, db = bat.scale_add_agg_weights_with_delta(wb, agg_b, n)
    wp = {k: v.to(DEV) for k, v in base0.items()}
    _, dp = per.scale_add_agg_weights_with_delta(wp, agg_p, n)
    wo = {k: v.clone() for k, v in base0.items()}
    do_ = {k: O.scale_add_tensor(wo[k], agg_o[k], n, want_delta=True) for k in wo}
    for lbl, a, b in (("agg", S.to_cpu(dict(agg_b)), S.to_cpu(dict(agg_p))), ("agg/oracle", S.to_cpu(dict(agg_b)), agg_o),
                      ("w", S.to_cpu(wb), S.to_cpu(wp)), ("w/oracle", S.to_cpu(wb), wo),
                      ("delta", S.to_cpu(db), S.to_cpu(dp)), ("delta/oracle", S.to_cpu(db), do_)):
        S.assert_bitwise(f"do_arrivals/{lbl}", a, b)


@pytest.mark.oracle
def test_hierarchy_round_from_batched_arrivals_vs_fixture(golden):
    """The reference-generated 2 x 3 hierarchy (hier_fedbuff_small.npz) with each middle's
    arrivals handed over in ONE FedBuff.do_arrivals call, then one hierarchy_round launch:
    top model and middle deltas bitwise == the reference's."""
    from flame_amd.optimizer.fedbuff import hierarchy_round
    fx = golden("hier_fedbuff_small.npz")
    rnd = fx.meta["round"]
    top_w0 = fx.weights("top_w0")
    mids = []
    for mid in range(2):
        arr = [S.TR({k: v.to(DEV) for k, v in fx.weights(f"m{mid}/update{t}").items()}, 10 + t, rnd - t % 2)
               for t in range(3)]
        agg = make_amd("fedbuff").do_arrivals(None, arr, version=rnd)
        mids.append(({k: v.to(DEV) for k, v in top_w0.items()}, agg, 3, rnd - mid))
    top = {k: v.to(DEV) for k, v in top_w0.items()}
    _, deltas = hierarchy_round(mids, None, version=rnd, top_weights=top, top_goal=2, with_delta=True)
    S.assert_bitwise("hier/top", S.to_cpu(top), fx.weights("top_out"))
    for mid in range(2):
        S.assert_bitwise(f"hier/delta m{mid}", S.to_cpu(deltas[mid]), fx.weights(f"m{mid}/delta"))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M", [4, 18])
def test_hierarchy_round_readonly_middles(dtype, M):
    """update_middle_weights=False (FLAME_HIER_MID_READONLY): middle weights untouched, the
    same tensor may serve every middle, and the top aggregate / top weights / deltas equal
    those of the in-place run with private copies, bitwise."""
    from flame_amd.optimizer.fedbuff import hierarchy_round
    g = torch.Generator().manual_seed(67)
    C, rnd, P = 3, 8, 5000
    ups = [[(torch.randn(P, generator=g) * 1e-2).to(dtype) for _ in range(C)] for _ in range(M)]
    fetched = torch.randn(P, generator=g).to(dtype)
    top0 = torch.randn(P, generator=g).to(dtype)

    def aggs():
        out = []
        for m in range(M):
            opt, a = make_amd("fedbuff"), None
            for t in range(C):
                cache = S.SortedCache()
                cache["a"] = S.TR({"x": ups[m][t].to(DEV)}, 1, rnd - (m + t) % 3)
                a = opt.do(a, cache, total=1, version=rnd)
            out.append(a)
        return out

    shared = fetched.to(DEV)
    tw_ro = {"x": top0.to(DEV)}
    agg_ro, d_ro = hierarchy_round([({"x": shared}, a, C, rnd - m % 2) for m, a in enumerate(aggs())], None,
                                   version=rnd, top_weights=tw_ro, top_goal=M, with_delta=True,
                                   update_middle_weights=False)
    own = [{"x": fetched.to(DEV)} for _ in range(M)]
    tw = {"x": top0.to(DEV)}
    agg, d = hierarchy_round([(own[m], a, C, rnd - m % 2) for m, a in enumerate(aggs())], None,
                             version=rnd, top_weights=tw, top_goal=M, with_delta=True)
    torch.cuda.synchronize()
    assert torch.equal(shared.cpu().view(torch.int16 if dtype != torch.float32 else torch.int32),
                       fetched.view(torch.int16 if dtype != torch.float32 else torch.int32))
    S.assert_bitwise("top agg", S.to_cpu(dict(agg_ro)), S.to_cpu(dict(agg)))
    S.assert_bitwise("top w", S.to_cpu(tw_ro), S.to_cpu(tw))
    for m in range(M):
        S.assert_bitwise(f"delta m{m}", S.to_cpu(d_ro[m]), S.to_cpu(d[m]))


def test_hierarchy_round_launch_count_and_fallback():
    """Uniform middles take ONE flame_hier_fedbuff launch per dtype; ragged arrival counts
    fall back to the separate launches with the same results; stale versions raise as
    FedBuff.do does (fedbuff.py:96)."""
    from flame_amd import engine
    from flame_amd.optimizer.fedbuff import hierarchy_round
    g = torch.Generator().manual_seed(43)
    rnd = 5

    def middles(counts):
        out = []
        for m, c in enumerate(counts):
            opt, agg = make_amd("fedbuff"), None
            for t in range(c):
                cache = S.SortedCache()
                cache["a"] = S.TR({"x": (torch.randn(777, generator=g) * 1e-2).to(DEV)}, 1, rnd - t % 2)
                agg = opt.do(agg, cache, total=1, version=rnd)
            out.append(({"x": torch.randn(777, generator=g).to(DEV)}, agg, c, rnd))
        return out

    engine.kernel_events = []
    try:
        hierarchy_round(middles([3, 3, 3]), None, version=rnd)
        names = [e[0] for e in engine.kernel_events]
        assert names == ["flame_hier_fedbuff"], names
        engine.kernel_events = []
        hierarchy_round(middles([3, 2]), None, version=rnd)
        names = [e[0] for e in engine.kernel_events]
        assert "flame_hier_fedbuff" not in names and "flame_fedbuff_scale_add" in names, names
    finally:
        engine.kernel_events = None
    mids = middles([2, 2])
    mids[1] = (mids[1][0], mids[1][1], 2, rnd + 1)
    with pytest.raises(ZeroDivisionError):
        hierarchy_round(mids, None, version=rnd)
    mids = middles([2, 2])
    mids[0] = ({"x": torch.zeros(776, device=DEV)}, mids[0][1], 2, rnd)   # weights / arrivals numel differ
    with pytest.raises((RuntimeError, NotImplementedError)):
        hierarchy_round(mids, None, version=rnd)


def test_metric_collector_receives_kernel_metrics():
    """optimizer.metric_collector gets runtime / hbm_GBps / launches per kernel of each call
    (saved once the kernels are done; metrics.flush() waits for them)."""
    from flame_amd import metrics

    class MC:
        def __init__(self):
            self.state_dict = {}

        def save(self, mtype, alias, value):
            self.state_dict[f"{alias}.{mtype}"] = value

    opt = make_amd("fedadam")
    opt.metric_collector = MC()
    g = torch.Generator().manual_seed(53)
    w = {"x": torch.randn(100_003, generator=g).to(DEV)}
    for rnd in range(2):
        cache = S.SortedCache()
        for i in range(4):
            cache[f"e{i}"] = S.TR({"x": (torch.randn(100_003, generator=g) * 1e-2).to(DEV)}, 10 + i)
        w = opt.do({k: v.clone() for k, v in w.items()}, cache, total=46)
    metrics.flush()
    sd = opt.metric_collector.state_dict
    assert sd["fedadam.flame_fedopt_reduce_adapt.launches"] == 1, sd
    assert sd["fedadam.flame_fedopt_reduce_adapt.runtime"] > 0
    assert sd["fedadam.flame_fedopt_reduce_adapt.hbm_GBps"] > 0


@pytest.mark.oracle
@pytest.mark.parametrize("where", ["zero_copy", "device_cache"])
def test_shm_receiver_registered_segment_to_fedavg(where):
    """LIFL SHM receive without host copies (flame_amd.ingest.ShmReceiver): each sender's
    segment is registered once; updates are either streamed by the kernel straight out of
    the shared segment or copied to HBM by DeviceUpdateCache; FedAvg bitwise == oracle."""
    import cloudpickle
    from multiprocessing import shared_memory
    from flame_amd import ingest
    O = _oracle()
    g = torch.Generator().manual_seed(59)
    n, P = 5, 70_001
    ws = [{"w": torch.randn(P, generator=g) * 1e-2} for _ in range(n)]
    counts = [20 + 3 * i for i in range(n)]
    segs, rx = [], ingest.ShmReceiver("agg", untrack=False)
    try:
        cache = ingest.DeviceUpdateCache(device=DEV, placement="hbm") if where == "device_cache" else S.SortedCache()
        for i, w in enumerate(ws):
            blob = cloudpickle.dumps({"weights": w, "dataset_size": counts[i]})
            seg = shared_memory.SharedMemory(name=f"flametest_t{i}-agg", create=True, size=len(blob))
            seg.buf[:len(blob)] = blob
            segs.append(seg)
            msg = rx.loads(f"flametest_t{i}", len(blob))
            assert msg["weights"]["w"].is_pinned()
            cache[f"t{i}"] = S.TR(msg["weights"], msg["dataset_size"])
            del msg
        base = torch.randn(P, generator=g)
        out = make_amd("fedavg").do({"w": base.to(DEV)}, cache, total=sum(counts))
        torch.cuda.synchronize()
        exp = base.clone()
        O.reduce_tensor(exp, [w["w"] for w in ws], [c / sum(counts) for c in counts])
        S.assert_bitwise("shm", S.to_cpu(out), {"w": exp})
        del cache, out
    finally:
        rx.close()
        for seg in segs:
            seg.close()
            seg.unlink()


@pytest.mark.oracle
def test_golden_nonfinite(golden):
    """nonfinite.npz, generated by the reference: the HIP path puts NaN and +-inf where the
    reference's torch-CPU ops do (FedAvg, FedBuff aggregate, FedBuff scale_add; f32 / bf16 /
    f16 / f64), every other element bitwise."""
    n = 0
    for label, got, exp in S.run_nonfinite(golden("nonfinite.npz"), make_amd, DEV):
        S.assert_same_nonfinite(f"nonfinite:{label}", got, exp)
        n += 1
    assert n == 12


@pytest.mark.oracle
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16, torch.float64])
def test_nonfinite_updates_match_oracle(dtype):
    """A diverged trainer (NaN, +-inf, overflowing sums): FedAvg and FedBuff + scale_add put
    NaN and +-inf exactly where the oracle (== the reference's torch-CPU ops) does, and
    every other element bitwise."""
    O = _oracle()
    base, cl, counts = S.nonfinite_case(dtype)
    tot = sum(counts)
    cache = S.SortedCache()
    for i, c in enumerate(cl):
        cache[f"e{i}"] = S.TR({"w": c.to(DEV)}, counts[i])
    got = make_amd("fedavg").do({"w": base.to(DEV)}, cache, total=tot)["w"]
    exp = base.clone()
    O.reduce_tensor(exp, cl, [c / tot for c in counts])
    assert torch.isnan(exp).sum() > 10 and torch.isinf(exp).sum() > 10
    S.assert_same_nonfinite(f"fedavg {dtype}", got, exp)
    if dtype == torch.float64:
        return
    fb, agg, ofb, oagg = make_amd("fedbuff"), None, O.OracleFedBuff(), None
    for i, c in enumerate(cl):
        c1, c2 = S.SortedCache(), S.SortedCache()
        c1["a"] = S.TR({"w": c.to(DEV)}, 1, 9 - i % 3)
        c2["a"] = S.TR({"w": c.clone()}, 1, 9 - i % 3)
        agg = fb.do(agg, c1, total=1, version=9)
        oagg = ofb.do(oagg, c2, total=1, version=9)
    w = {"w": base.to(DEV)}
    fb.scale_add_agg_weights(w, agg, len(cl))
    ow = {"w": base.clone()}
    ofb.scale_add_agg_weights(ow, oagg, len(cl))
    S.assert_same_nonfinite(f"fedbuff {dtype}", w["w"], ow["w"])


@pytest.mark.oracle
@pytest.mark.parametrize("with_delta,slab", [(True, False), (False, False), (True, True)])
def test_sync_hierarchy_golden(golden, with_delta, slab):
    """sync_hierarchy_round (one FLAME_HIER_SYNC launch per float dtype; the int64 key
    composes the separate calls) == the reference's syncfl middles + top, bitwise
    (hier_fedavg_small.npz: 3 middles x 4 trainers, f32/bf16/f16/int64, 2 rounds)."""
    from flame_amd import engine
    launches = []
    engine._recorders.append(launches)
    try:
        res = S.run_hier_fedavg_fused(golden("hier_fedavg_small.npz"), DEV, with_delta=with_delta, slab=slab)
    finally:
        engine._recorders.remove(launches)
    for label, got, exp in res:
        S.assert_bitwise(f"hier_fedavg:{label}", got, exp)
    assert sum(1 for ev in launches if ev[0] == "flame_hier_fedbuff") == 3 * 2   # f32, bf16, f16 x 2 rounds


@pytest.mark.oracle
@pytest.mark.parametrize("M", [8, 20])
@pytest.mark.parametrize("path", ["argmeta", "table"])
def test_sync_hierarchy_vs_oracle_readonly_middles(M, path, monkeypatch):
    """8 / 20 middles x 16 trainers over ~1M params (tails, every float dtype + int64): top
    and deltas == the oracle's FedAvg / delta / FedAvg composition; with
    update_middle_weights=False one shared middle tensor is read, never written.  20
    middles take the LDS-held store groups (a full group of 16 + 4).  Both metadata paths."""
    from flame_amd import engine
    from flame_amd.optimizer.sync_hierarchy import sync_hierarchy_round
    O = _oracle()
    if path == "table":
        monkeypatch.setattr(engine, "ARGMETA", False)
    g = torch.Generator().manual_seed(41)
    tmpl = _dyn_model(g, 1_000_003)
    C = 16
    mid_cpu = {k: v.clone() for k, v in tmpl.items()}
    top_cpu = {k: (v * 0.5 if v.is_floating_point() else v) for k, v in tmpl.items()}
    ups = [[_dyn_update(g, tmpl, 5 * j + i) for i in range(C)] for j in range(M)]
    counts = [[int(x) for x in torch.randint(1, 1000, (C,), generator=g)] for _ in range(M)]
    shared = {k: v.to(DEV) for k, v in mid_cpu.items()}
    specs = []
    for j in range(M):
        cache = S.SortedCache()
        for i in range(C):
            cache[f"m{j}t{i:02d}"] = S.TR({k: v.to(DEV) for k, v in ups[j][i].items()}, counts[j][i])
        specs.append((shared, cache, sum(counts[j])))
    top = {k: v.to(DEV) for k, v in top_cpu.items()}
    top, deltas = sync_hierarchy_round(specs, top, with_delta=True, update_middle_weights=False)
    S.assert_bitwise("sync/readonly/middle", S.to_cpu(shared), mid_cpu)
    # oracle: the separate calls
    exp_deltas, top_cache = [], S.SortedCache()
    for j in range(M):
        cache = S.SortedCache()
        for i in range(C):
            cache[f"m{j}t{i:02d}"] = S.TR({k: v.clone() for k, v in ups[j][i].items()}, counts[j][i])
        new = O.OracleFedAvg().do({k: v.clone() for k, v in mid_cpu.items()}, cache, total=sum(counts[j]))
        exp_deltas.append({k: new[k] - mid_cpu[k] for k in new})
        top_cache[f"mid{j:02d}"] = S.TR(exp_deltas[-1], sum(counts[j]))
    exp_top = O.OracleFedAvg().do({k: v.clone() for k, v in top_cpu.items()}, top_cache,
                                  total=sum(sum(c) for c in counts))
    for j in range(M):
        S.assert_bitwise(f"sync/readonly/delta{j}", S.to_cpu(deltas[j]), exp_deltas[j])
    S.assert_bitwise("sync/readonly/top", S.to_cpu(top), exp_top)


def _sharded_opt_gpu_worker(rank, world, port, q):
    import os
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)   # two ranks share the one GPU
    ok = True
    try:
        from flame_amd import shard
        from flame_amd.optimizers import optimizer_provider
        from flame_amd.slab import UpdateSlab
        g = torch.Generator().manual_seed(51)
        tmpl = _dyn_model(g, 300_007)
        hyper = dict(beta_1=0.9, beta_2=0.99, eta=1e-2, tau=1e-3)
        sharded = shard.ShardedOptimizer(optimizer_provider.get("fedadam", **hyper))
        single = optimizer_provider.get("fedadam", **hyper)
        slab = UpdateSlab({k: v for k, v in tmpl.items()}, capacity=16, device=DEV)
        ws = {k: v.to(DEV) for k, v in tmpl.items()}
        wr = {k: v.clone() for k, v in ws.items()}
        for r in range(3):
            ups = [_dyn_update(g, tmpl, 3 * r + i) for i in range(6)]
            counts = [11 + 7 * i for i in range(6)]
            ca, cb = S.SortedCache(), S.SortedCache()
            for i, u in enumerate(ups):
                ca[f"t{i}"] = S.TR(slab.put({k: v.to(DEV) for k, v in u.items()}), counts[i])
                cb[f"t{i}"] = S.TR({k: v.to(DEV) for k, v in u.items()}, counts[i])
            ws = sharded.do({k: v.clone() for k, v in ws.items()}, ca, total=sum(counts))
            wr = single.do({k: v.clone() for k, v in wr.items()}, cb, total=sum(counts))
            torch.cuda.synchronize()
            for k in wr:
                a, b = ws[k].cpu(), wr[k].cpu()
                ok = ok and a.dtype == b.dtype and torch.equal(a.view(torch.int16) if a.dtype in (torch.bfloat16, torch.half) else a,
                                                               b.view(torch.int16) if b.dtype in (torch.bfloat16, torch.half) else b)
            del ca, cb
        q.put((rank, bool(ok)))
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def test_sharded_fedadam_two_ranks_one_gpu():
    """ShardedOptimizer(FedAdam drop-in) with two gloo ranks sharing the GPU: each rank runs
    the HIP FedAdam on its per-key slices of slab-resident updates (tiled views sliced
    tiled); the gathered model == one process's FedAdam, bitwise, over 3 rounds (f32, bf16,
    f16 keys and an int64 buffer that FedOPT promotes)."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_sharded_opt_gpu_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=100) for _ in ps)
    for p in ps:
        p.join(timeout=30)
    assert res == {0: True, 1: True}, res


@pytest.mark.oracle
@pytest.mark.parametrize("variant", ["fedadam", "fedyogi", "fedadagrad"])
def test_c4_full_size_every_element(variant):
    """Config 4 at full size (FedAdam / FedYogi / FedAdaGrad, 1024 x 25M fp32 in a tiled slab, round 1
    passthrough then an adaptive round; fedadam.py:33-35, fedyogi.py:34-36, fedadagrad.py:33-35,
    fedopt.py:58-129), EVERY element vs the C oracle: round 1's result and the adaptive round's
    average bitwise, its cur / m / v within the §8(c) contract (the oracle's sqrt is correctly
    rounded like the kernel's; the count of bit-equal elements is reported)."""
    import full_check as F
    from flame_amd import synth, engine
    from flame_amd.slab import UpdateSlab
    O = _oracle()
    n, P = 1024, 25_000_000
    free, _ = torch.cuda.mem_get_info()
    if free < (n + 10) * P * 4:
        pytest.skip(f"needs {(n + 10) * P * 4 / 1e9:.1f} GB of HBM, {free / 1e9:.1f} GB free")
    slab = UpdateSlab({"model": torch.empty(P)}, capacity=n, device=DEV)
    tmp = torch.empty(P, device=DEV)
    ws = []
    for i in range(n):
        engine.synth_fill_(tmp, 3, 1 + i, 0, 1e-2)
        ws.append(slab.put({"model": tmp}))
    del tmp
    base = _synth_dev(3, 0, P, 1.0)
    base0 = base.cpu().numpy()
    hyper = dict(beta_1=0.9, beta_2=0.99, eta=1e-2, tau=1e-3)
    amd = make_amd(variant, **hyper)
    rates, outs = [], []
    wa = {"model": base}
    for r in range(2):
        counts = synth.counts(3 + r, n)
        total = int(counts.sum())
        rates.append([int(c) / total for c in counts])
        ca = S.SortedCache()
        for i in range(n):
            ca[f"{i:05d}"] = S.TR(ws[i], int(counts[i]))
        wa = amd.do({"model": wa["model"].clone()}, ca, total=total)
        outs.append(wa["model"].cpu().numpy())
    avg1 = amd.agg_weights["model"].cpu().numpy()
    m1, v1 = amd.m_t["model"].cpu().numpy(), amd.v_t["model"].cpu().numpy()
    cur1 = outs[1]
    r0 = [float(x) for x in O.fedopt_scalars(**hyper)]
    bad0 = bad_avg = eq = 0
    worst = [0.0, 0.0, 0.0]
    l2 = {k: [0.0, 0.0] for k in ("cur", "m", "v")}
    for e0, e1, host in F.columns(slab.storage[torch.float32], n, P):
        acc = base0[e0:e1].copy()
        F.reduce_chunk(host, acc, rates[0], torch.float32)          # round 1: FedAvg, current := avg
        bad0 += F.mismatches(acc, outs[0][e0:e1])
        cur0 = acc.copy()
        F.reduce_chunk(host, acc, rates[1], torch.float32)          # round 2: FedAvg from current ...
        bad_avg += F.mismatches(acc, avg1[e0:e1])
        m = np.zeros(e1 - e0, np.float32)
        v = np.zeros(e1 - e0, np.float32)
        cur = F.fedopt_adapt(variant, acc, cur0, m, v, r0)          # ... then the adaptive step (state None)
        for j, (lbl, got, ref) in enumerate((("cur", cur1[e0:e1], cur), ("m", m1[e0:e1], m), ("v", v1[e0:e1], v))):
            el, _ = F.close_fedopt(got, ref)
            worst[j] = max(worst[j], el)
            l2[lbl][0] += float(np.sum((got.astype(np.float64) - ref) ** 2))
            l2[lbl][1] += float(np.sum(ref.astype(np.float64) ** 2))
        eq += (e1 - e0) - F.mismatches(cur1[e0:e1], cur)
    assert bad0 == 0 and bad_avg == 0, (bad0, bad_avg)
    rel = {k: (a / b) ** 0.5 if b else 0.0 for k, (a, b) in l2.items()}
    assert max(worst) <= 1e-6 and max(rel.values()) <= 1e-6, (worst, rel)
    print(f"c4/{variant}: every element checked; cur bit-equal to the C oracle on {eq} of {P}; "
          f"max elementwise rel err cur/m/v {worst}, rel-L2 {rel}")
    del ws, slab, wa, amd
    torch.cuda.empty_cache()


@pytest.mark.oracle
def test_c5_full_size_hierarchy_every_element():
    """Config 5's per-GPU shard at full size (64 middles x 64 arrivals x 15.625M bf16 = 128 GB
    in a tiled slab, staleness 0..3): ONE hierarchy_round launch; EVERY element of every
    middle's new weights, of the top aggregate and of the top weights == the C oracle's FedBuff
    op sequence (per-arrival do with a None start, scale_add + delta per middle, the top's do per
    delta, the top's scale_add; fedbuff.py:59-157, asyncfl/middle_aggregator.py:164-246,
    asyncfl/top_aggregator.py:85-110), bitwise."""
    import collections
    import full_check as F
    from flame_amd import synth, engine
    from flame_amd.optimizer.fedbuff import hierarchy_round
    from flame_amd.slab import UpdateSlab
    M, C, P, rnd = 64, 64, 15_625_000, 10
    free, _ = torch.cuda.mem_get_info()
    if free < (M * C + 2 * M + 8) * P * 2:
        pytest.skip(f"needs {(M * C + 2 * M + 8) * P * 2 / 1e9:.1f} GB of HBM, {free / 1e9:.1f} GB free")
    dt = torch.bfloat16
    slab = UpdateSlab({"model": torch.empty(P, dtype=dt)}, capacity=M * C, device=DEV)
    tmp = torch.empty(P, dtype=dt, device=DEV)
    ws = []
    for i in range(M * C):
        engine.synth_fill_(tmp, 6, 1 + i, 0, 1e-2)
        ws.append(slab.put({"model": tmp}))
    mids = []
    for m in range(M):
        engine.synth_fill_(tmp, 6, 10_000 + m, 0, 1.0)
        mids.append(tmp.clone())
    engine.synth_fill_(tmp, 6, 0, 0, 1.0)
    top_w = tmp.clone()
    del tmp
    mids0 = [F.bits(x) for x in mids]            # the middles' weights before the round (host)
    top0 = F.bits(top_w)
    stale = [int(x) % 4 for x in synth.counts(6, M * C)]
    aggs = [make_amd("fedbuff").do_arrivals(None, [S.TR(ws[m * C + t], 1, rnd - stale[m * C + t]) for t in range(C)],
                                            version=rnd) for m in range(M)]
    top_agg, _ = hierarchy_round([({"model": mids[m]}, aggs[m], C, rnd - (m % 2)) for m in range(M)], None,
                                 version=rnd, top_weights={"model": top_w}, top_goal=M)
    torch.cuda.synchronize()
    top_agg_g, top_w_g = F.bits(top_agg["model"]), F.bits(top_w)
    mid_rates = [[1 / math.sqrt(1 + stale[m * C + t]) for t in range(C)] for m in range(M)]
    top_rates = [1 / math.sqrt(1 + m % 2) for m in range(M)]
    bad = collections.Counter()
    checked = 0
    for e0, e1, host in F.columns(slab.storage[dt], M * C, P, chunk_tiles=64):
        top = np.empty(e1 - e0, np.uint16)
        for m in range(M):
            agg = np.empty(e1 - e0, np.uint16)
            F.reduce_chunk(host[m * C:m * C + 1], agg, mid_rates[m][:1], dt, init_first=True)   # None start
            F.reduce_chunk(host[m * C + 1:(m + 1) * C], agg, mid_rates[m][1:], dt)
            w = mids0[m][e0:e1].copy()
            delta = F.scale_add(w, agg, C, dt, want_delta=True)
            bad["mid"] += F.mismatches(w, F.bits(mids[m][e0:e1]))
            F.reduce_chunk(torch.from_numpy(delta.view(np.int16)).view(dt).view(1, -1), top, top_rates[m:m + 1], dt,
                           init_first=(m == 0))
        bad["top agg"] += F.mismatches(top, top_agg_g[e0:e1])
        tw = top0[e0:e1].copy()
        F.scale_add(tw, top, M, dt)
        bad["top w"] += F.mismatches(tw, top_w_g[e0:e1])
        checked += e1 - e0
    assert checked == P and not +bad, dict(bad)
    del ws, aggs, slab, top_agg
    torch.cuda.empty_cache()



def test_mnist_example_config1():
    """Config 1 (examples/mnist: 2 trainers x MNIST Net, counts 2000/2000) end to end through
    channel payloads -> ingest.decode -> DeviceUpdateCache -> FedAvg drop-in, bitwise vs the
    reference's op sequence each round (examples/mnist_aggregation.py)."""
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location(
        "mnist_aggregation", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                          "examples", "mnist_aggregation.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    assert mod.run(rounds=3, verbose=False)


@pytest.mark.oracle
def test_integration_ctypes_stub_runs():
    """The reference-side ctypes stub printed in INTEGRATION.md §2 works as written
    (library path substituted) and equals the oracle's FedAvg, bitwise."""
    import os
    import re
    from flame_amd import _native
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    doc = open(os.path.join(root, "INTEGRATION.md")).read()
    code = re.search(r"```python\n(# flame/optimizer/_mi355x\.py.*?)```", doc, re.S).group(1)
    code = code.replace('ctypes.CDLL("libflame_amd.so")', f'ctypes.CDLL("{_native.LIB_PATH}")')
    ns = {}
    exec(compile(code, "INTEGRATION.md:stub", "exec"), ns)
    O = _oracle()
    g = torch.Generator().manual_seed(77)
    P, n = 100_003, 9
    agg = torch.randn(P, generator=g)
    ups = [torch.randn(P, generator=g) * 1e-2 for _ in range(n)]
    rates = [(i + 1) / 45 for i in range(n)]
    dev_agg = agg.to(DEV)
    ns["aggregate_fp32"](dev_agg, [u.to(DEV) for u in ups], rates)
    torch.cuda.synchronize()
    exp = agg.clone()
    O.reduce_tensor(exp, ups, rates)
    S.assert_bitwise("ctypes stub", {"x": dev_agg}, {"x": exp})


@pytest.mark.oracle
def test_empty_and_tiny_keys_every_path():
    """Models with 0-element and 1-element tensors between ordinary ones: FedAvg, FedAdam,
    FedBuff (fused scale_add), FedDyn and the sync hierarchy all match the oracle, bitwise
    (FedOPT within the §8(c) contract)."""
    from flame_amd.optimizer.sync_hierarchy import sync_hierarchy_round
    O = _oracle()
    g = torch.Generator().manual_seed(91)
    shapes = {"a": (0,), "w": (5000,), "e": (0, 7), "one": (1,), "m": (33, 3)}

    def model(scale):
        return {k: torch.randn(s, generator=g) * scale for k, s in shapes.items()}
    base, ups = model(1.0), [model(1e-2) for _ in range(5)]
    counts = [3, 9, 1, 4, 7]

    def caches():
        ca, co = S.SortedCache(), S.SortedCache()
        for i, (u, c) in enumerate(zip(ups, counts)):
            ca[f"t{i}"] = S.TR({k: v.to(DEV) for k, v in u.items()}, c, 5 - i % 2)
            co[f"t{i}"] = S.TR({k: v.clone() for k, v in u.items()}, c, 5 - i % 2)
        return ca, co
    # FedAvg
    ca, co = caches()
    out = make_amd("fedavg").do({k: v.to(DEV) for k, v in base.items()}, ca, total=sum(counts))
    exp = O.OracleFedAvg().do({k: v.clone() for k, v in base.items()}, co, total=sum(counts))
    S.assert_bitwise("fedavg", S.to_cpu(out), exp)
    # FedAdam: passthrough round then an adaptive round
    amd, ora = make_amd("fedadam"), O.OracleFedOPT("fedadam")
    wa, wo = {k: v.to(DEV) for k, v in base.items()}, {k: v.clone() for k, v in base.items()}
    for _ in range(2):
        ca, co = caches()
        wa = amd.do({k: v.clone() for k, v in wa.items()}, ca, total=sum(counts))
        wo = ora.do({k: v.clone() for k, v in wo.items()}, co, total=sum(counts))
    S.assert_close_fedopt("fedadam", S.to_cpu(wa), wo)
    # FedBuff: arrivals one per do(), fused scale_add
    fb, ob, fa, oa = make_amd("fedbuff"), O.OracleFedBuff(), None, None
    for i, (u, c) in enumerate(zip(ups, counts)):
        c1, c2 = S.SortedCache(), S.SortedCache()
        c1["a"] = S.TR({k: v.to(DEV) for k, v in u.items()}, c, 5 - i % 2)
        c2["a"] = S.TR({k: v.clone() for k, v in u.items()}, c, 5 - i % 2)
        fa = fb.do(fa, c1, total=c, version=5)
        oa = ob.do(oa, c2, total=c, version=5)
    wb, wbo = {k: v.to(DEV) for k, v in base.items()}, {k: v.clone() for k, v in base.items()}
    fb.scale_add_agg_weights(wb, fa, 5)
    ob.scale_add_agg_weights(wbo, oa, 5)
    S.assert_bitwise("fedbuff", S.to_cpu(wb), wbo)
    # FedDyn, two rounds
    da, do_ = make_amd("feddyn", alpha=0.1), O.OracleFedDyn(alpha=0.1)
    xa, xo = {k: v.to(DEV) for k, v in base.items()}, {k: v.clone() for k, v in base.items()}
    for _ in range(2):
        da.save_state(S._PRE, active_ends=[f"t{i}" for i in range(5)])
        do_.save_state(S._PRE, active_ends=[f"t{i}" for i in range(5)])
        ca, co = caches()
        xa = da.do({k: v.clone() for k, v in xa.items()}, ca, total=sum(counts))
        xo = do_.do({k: v.clone() for k, v in xo.items()}, co, total=sum(counts))
        S.assert_bitwise("feddyn cld", S.to_cpu(da.cld_model), do_.cld_model)
        xa, xo = da.cld_model, do_.cld_model
    # sync hierarchy: two middles of the same five trainers
    mids = [{k: v.to(DEV) for k, v in base.items()} for _ in range(2)]
    top = {k: v.to(DEV) for k, v in base.items()}
    specs = [(mids[j], caches()[0], sum(counts)) for j in range(2)]
    top, _ = sync_hierarchy_round(specs, top)
    exp_mid = O.OracleFedAvg().do({k: v.clone() for k, v in base.items()}, caches()[1], total=sum(counts))
    d = {k: exp_mid[k] - base[k] for k in base}
    tc = S.SortedCache()
    tc["m0"], tc["m1"] = S.TR(d, sum(counts)), S.TR({k: v.clone() for k, v in d.items()}, sum(counts))
    exp_top = O.OracleFedAvg().do({k: v.clone() for k, v in base.items()}, tc, total=2 * sum(counts))
    S.assert_bitwise("sync mid", S.to_cpu(mids[0]), exp_mid)
    S.assert_bitwise("sync top", S.to_cpu(top), exp_top)


@pytest.mark.oracle
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16, torch.float64, torch.int64])
def test_argmeta_launch_equals_device_table_launch(dtype):
    """Small launches pass the metadata as a kernel argument (flame_agg_reduce_argmeta); the
    result equals the device-table launch and the oracle, bitwise -- plain, INIT_FIRST and
    per-segment rate rows (FLAME_AGG_SEG_RATES) -- and big tables still take the upload path."""
    from flame_amd import engine
    O = _oracle()
    g = torch.Generator().manual_seed(93)
    shapes = [(5000,), (3, 77), (1,), (0,), (2049,)]

    def rnd(s, scale):
        x = torch.randn(s, generator=g, dtype=torch.float64) * scale
        return (x * 1000).to(dtype) if dtype == torch.int64 else x.to(dtype)
    n = 7
    base = [rnd(s, 1.0) for s in shapes]
    cl = [[rnd(s, 1e-2) for _ in range(n)] for s in shapes]
    rates = [(i + 2) / 37 for i in range(n)]
    rows = [[(i + 1 + j) / 41 for i in range(n)] for j in range(len(shapes))]
    results = {}
    for argmeta in (True, False):
        engine.ARGMETA = argmeta
        try:
            outs = [b.to(DEV) for b in base]
            engine.reduce_(outs, outs, [[c.to(DEV) for c in row] for row in cl], rates)
            first = [torch.empty(b.shape, dtype=dtype, device=DEV) for b in base]
            engine.reduce_(first, None, [[c.to(DEV) for c in row] for row in cl], rates, init_first=True)
            segr = [b.to(DEV) for b in base]
            engine.reduce_(segr, segr, [[c.to(DEV) for c in row] for row in cl], None, seg_rates=rows)
            torch.cuda.synchronize()
            results[argmeta] = [[t.cpu() for t in ts] for ts in (outs, first, segr)]
        finally:
            engine.ARGMETA = True
    for a, b in zip(results[True], results[False]):
        for j, (x, y) in enumerate(zip(a, b)):
            S.assert_bitwise(f"argmeta/{dtype}/{j}", {"x": x}, {"x": y})
    for j, b in enumerate(base):
        exp = b.clone()
        O.reduce_tensor(exp, cl[j], rates)
        S.assert_bitwise(f"oracle/{dtype}/{j}", {"x": results[True][0][j]}, {"x": exp})


@pytest.mark.oracle
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_many_clients_one_launch(dtype):
    """The largest flat reduction the BASELINE configs imply: all 4096 clients of config 5
    (+1, an odd count) in ONE FedAvg launch over three keys (ragged sizes, one empty),
    read from a tiled slab -- bitwise vs the oracle; and 4096 FedBuff arrivals queued then
    read once (one launch) equal the oracle's per-arrival sequence."""
    from flame_amd.slab import UpdateSlab
    O = _oracle()
    n = 4097
    shapes = {"a": (3000,), "b": (7,), "c": (0,)}
    g = torch.Generator().manual_seed(4097)
    base = {k: torch.randn(s, generator=g, dtype=torch.float64).to(dtype) for k, s in shapes.items()}
    cl = [{k: (torch.randn(s, generator=g, dtype=torch.float64) * 1e-2).to(dtype) for k, s in shapes.items()}
          for _ in range(n)]
    counts = torch.randint(1, 1000, (n,), generator=g).tolist()
    total = sum(counts)
    exp = {k: v.clone() for k, v in base.items()}
    for k in shapes:
        O.reduce_tensor(exp[k], [c[k] for c in cl], [c / total for c in counts])
    slab = UpdateSlab(base, capacity=n, device=DEV)
    cache = S.SortedCache()
    for i, (c, k) in enumerate(zip(cl, counts)):
        cache[f"{i:05d}"] = S.TR(slab.put({kk: v.to(DEV) for kk, v in c.items()}), k)
    from flame_amd import engine
    engine.kernel_events = []
    try:
        out = make_amd("fedavg").do({k: v.to(DEV) for k, v in base.items()}, cache, total=total)
        assert len(engine.kernel_events) == 1, [e[0] for e in engine.kernel_events]
    finally:
        engine.kernel_events = None
    S.assert_bitwise(f"fedavg {n} clients {dtype}", out, exp)
    del slab, cache
    # FedBuff: 4096 queued arrivals, staleness 0..3, into an existing aggregate
    m = 4096
    vers = torch.randint(0, 4, (m,), generator=g).tolist()
    agg0 = {k: (torch.randn(s, generator=g, dtype=torch.float64) * 1e-2).to(dtype) for k, s in shapes.items()}
    exp = {k: v.clone() for k, v in agg0.items()}
    rates = [1 / math.sqrt(1 + 3 - v) for v in vers]
    for k in shapes:
        O.reduce_tensor(exp[k], [c[k] for c in cl[:m]], rates)
    opt = make_amd("fedbuff")
    agg = {k: v.to(DEV) for k, v in agg0.items()}
    for i in range(m):
        cache = S.SortedCache()
        cache[f"{i:05d}"] = S.TR({k: v.to(DEV) for k, v in cl[i].items()}, 1, vers[i])
        agg = opt.do(agg, cache, total=1, version=3)
    S.assert_bitwise(f"fedbuff {m} arrivals {dtype}", {k: agg[k] for k in shapes}, exp)


@pytest.mark.oracle
@pytest.mark.parametrize("sort", ["fedadam", "fedyogi", "fedadagrad"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_fedopt_argmeta_equals_device_table(sort, dtype):
    """Small FedOPT rounds pass their metadata as a kernel argument
    (flame_fedopt_reduce_adapt_argmeta); with engine.ARGMETA off they take the device-table
    launch (flame_fedopt_reduce_adapt, one chunk per workgroup).  Three rounds (passthrough,
    zero state, running state): the two launches equal each other bitwise, and each round of
    both equals OracleFedOPT.do (fedopt.py:58-129) from the same state at the round's start --
    the average bitwise, current / m / v within the §8(c) contract (fp32) or bitwise (bf16: every
    op rounded to bf16, as the reference's torch-CPU ops round it)."""
    from flame_amd import engine
    O = _oracle()
    g = torch.Generator().manual_seed(17)
    shapes = {"w": (300, 7), "b": (7,), "e": (0,), "t": (4099,)}
    w0 = {k: torch.randn(s, generator=g, dtype=torch.float64).to(dtype) for k, s in shapes.items()}
    rounds = [[({k: (w0[k].double() + torch.randn(s, generator=g, dtype=torch.float64) * 1e-2).to(dtype)
                 for k, s in shapes.items()}, int(c)) for c in torch.randint(1, 500, (5,), generator=g)]
              for _ in range(3)]
    from flame_amd import _native
    dt = {torch.float32: "f32", torch.bfloat16: "bf16"}[dtype]
    results = {}
    for argmeta in (True, False):
        engine.ARGMETA = argmeta
        before = _native.launch_branch_counts()
        try:
            opt = make_amd(sort)
            w = {k: v.to(DEV) for k, v in w0.items()}
            outs = []
            for arrivals in rounds:
                cache = S.SortedCache()
                for i, (u, c) in enumerate(arrivals):
                    cache[f"{i:03d}"] = S.TR({k: v.to(DEV) for k, v in u.items()}, c)
                w = opt.do({k: v.clone() for k, v in w.items()}, cache, total=sum(c for _, c in arrivals))
                outs.append([S.to_cpu(dict(x)) if x is not None else None
                             for x in (w, opt.agg_weights, opt.m_t, opt.v_t)])
            results[argmeta] = outs
        finally:
            engine.ARGMETA = True
        after = _native.launch_branch_counts()
        hits = {k: after[k] - before.get(k, 0) for k in after
                if after[k] != before.get(k, 0) and k.startswith("flame_fedopt")}
        want = f"flame_fedopt_reduce_adapt{'_argmeta' if argmeta else ''}/{dt}/{sort}"
        assert hits == {want: 2}, hits          # rounds 2 and 3 (round 1 is the passthrough)
    for r, (a, b) in enumerate(zip(results[True], results[False])):
        for lbl, x, y in zip(("cur", "avg", "m", "v"), a, b):
            if y is not None:
                S.assert_bitwise(f"{sort}/{dtype}/round{r}/{lbl}", x, y)
    ulp = 2.0 ** -7
    for argmeta, outs in results.items():
        ora = O.OracleFedOPT(sort)
        prev = {k: v.clone() for k, v in w0.items()}
        for r, arrivals in enumerate(rounds):
            if r >= 1:
                ora.current_weights = {k: v.clone() for k, v in outs[r - 1][0].items()}
            if r >= 2:
                ora.m_t = {k: v.clone() for k, v in outs[r - 1][2].items()}
                ora.v_t = {k: v.clone() for k, v in outs[r - 1][3].items()}
            cache = S.SortedCache()
            for i, (u, c) in enumerate(arrivals):
                cache[f"{i:03d}"] = S.TR({k: v.clone() for k, v in u.items()}, c)
            exp = ora.do({k: v.clone() for k, v in prev.items()}, cache, total=sum(c for _, c in arrivals))
            cur, avg, m, v = outs[r]
            lbl = f"oracle/{sort}/{dtype}/argmeta={argmeta}/round{r}"
            S.assert_bitwise(f"{lbl}/avg", avg, ora.agg_weights)
            for name, x, y in (("cur", cur, exp), ("m", m, ora.m_t), ("v", v, ora.v_t)):
                if r == 0 and name != "cur":
                    assert x is None and y is None, (lbl, name)
                    continue
                if dtype == torch.float32:
                    S.assert_close_fedopt(f"{lbl}/{name}", x, y)
                else:
                    for k in y:
                        gg, ee = x[k].double(), y[k].double()
                        bad = ((gg - ee).abs() > ee.abs() * ulp + 1e-30).nonzero().flatten()
                        assert bad.numel() == 0, f"{lbl}/{name}/{k}: {bad.numel()} beyond one ulp"
                    S.assert_bitwise(f"{lbl}/{name}", x, y)
            prev = {k: t.clone() for k, t in cur.items()}


@pytest.mark.parametrize("sort", ["fedadam", "fedyogi", "fedadagrad"])
@pytest.mark.parametrize("case", ["f32_slab", "bf16_slab", "f16_tensors", "f32_big"])
def test_fedopt_split_launch_equals_fused(sort, case):
    """FedOPT.split_launch (the FedAvg reduction, then the adaptive step as a no-client
    flame_fedopt_reduce_adapt) == the one fused launch, bitwise: avg, cur, m, v over three
    rounds (passthrough, zero state, running state).  f32_big takes the multi-chunk workgroup
    path (FLAME_OPT_WGC) of the fused kernel."""
    from flame_amd.optimizer.fedopt import FedOPT
    from flame_amd.slab import UpdateSlab
    dtype = {"f32_slab": torch.float32, "bf16_slab": torch.bfloat16, "f16_tensors": torch.float16,
             "f32_big": torch.float32}[case]
    g = torch.Generator().manual_seed(23)
    shapes = {"w": (20_000_000,)} if case == "f32_big" else {"w": (300, 7), "b": (7,), "t": (4099,)}
    n = 3 if case == "f32_big" else 6
    w0 = {k: torch.randn(sh, generator=g).to(dtype) for k, sh in shapes.items()}
    rounds = [[({k: (torch.randn(sh, generator=g) * 1e-2).to(dtype) for k, sh in shapes.items()}, 10 + 7 * i)
               for i in range(n)] for _ in range(3)]
    results = {}
    for split in (False, True):
        FedOPT.split_launch = split
        try:
            opt = make_amd(sort)
            slab = UpdateSlab({k: torch.empty(sh, dtype=dtype) for k, sh in shapes.items()}, capacity=n, device=DEV) \
                if case.endswith("slab") else None
            w = {k: v.to(DEV) for k, v in w0.items()}
            outs = []
            for arrivals in rounds:
                cache = S.SortedCache()
                for i, (u, c) in enumerate(arrivals):
                    ud = {k: v.to(DEV) for k, v in u.items()}
                    cache[f"{i:03d}"] = S.TR(slab.put(ud) if slab is not None else ud, c)
                w = opt.do({k: v.clone() for k, v in w.items()}, cache, total=sum(c for _, c in arrivals))
                outs.append([S.to_cpu(dict(x)) for x in (w, opt.agg_weights, opt.m_t or {}, opt.v_t or {})])
            results[split] = outs
        finally:
            FedOPT.split_launch = False
    for r, (a, b) in enumerate(zip(results[False], results[True])):
        for lbl, x, y in zip(("cur", "avg", "m", "v"), a, b):
            S.assert_bitwise(f"{sort}/{case}/round{r}/{lbl}", x, y)


@pytest.mark.oracle
def test_key_subset_arrivals():
    """Updates carrying a SUBSET of the model's keys (fedavg.py:93 / fedbuff.py:143 add
    ``for k, v in tres.weights.items()``: a key a client did not send keeps its value).
    FedAvg and FedBuff bitwise vs the oracle -- FedBuff's deferred None-start aggregate
    with later arrivals lacking keys included -- FedAdam within the §8(c) tolerance; an
    update naming a key the aggregate lacks raises KeyError like the reference's
    ``agg[k] += tmp``."""
    O = _oracle()
    g = torch.Generator().manual_seed(2024)
    shapes = {"a": ((1000,), torch.float32), "b": ((37,), torch.bfloat16), "n": ((3,), torch.int64)}

    def rnd(k, scale=1.0):
        s, dt = shapes[k]
        if dt == torch.int64:
            return torch.randint(0, 50, s, generator=g)
        return (torch.randn(s, generator=g, dtype=torch.float64) * scale).to(dt)

    subsets = [("a", "b", "n"), ("a", "n"), ("b",), ("a", "b")]
    base = {k: rnd(k) for k in shapes}
    cl = [{k: rnd(k, 1e-2) for k in ks} for ks in subsets]
    counts = [3, 5, 7, 11]
    total = sum(counts)

    def cache_of(ws, cnts, vers=None):
        c = S.SortedCache()
        for i, (w, n) in enumerate(zip(ws, cnts)):
            c[f"{i:03d}"] = S.TR({k: v.to(DEV) for k, v in w.items()}, n, 0 if vers is None else vers[i])
        return c

    def cpu_cache(ws, cnts, vers=None):
        c = S.SortedCache()
        for i, (w, n) in enumerate(zip(ws, cnts)):
            c[f"{i:03d}"] = S.TR({k: v.clone() for k, v in w.items()}, n, 0 if vers is None else vers[i])
        return c

    # FedAvg
    got = make_amd("fedavg").do({k: v.to(DEV) for k, v in base.items()}, cache_of(cl, counts), total=total)
    exp = O.OracleFedAvg().do({k: v.clone() for k, v in base.items()}, cpu_cache(cl, counts), total=total)
    S.assert_bitwise("fedavg subsets", got, exp)

    # FedBuff: None-start from the full arrival, then subset arrivals, one do() each; scale_add
    vers = [2, 1, 0, 2]
    for defer in (True, False):
        opt, ref = make_amd("fedbuff", defer=defer), O.OracleFedBuff()
        agg = eagg = None
        for i in range(len(cl)):
            agg = opt.do(agg, cache_of([cl[i]], [1], [vers[i]]), total=1, version=2)
            eagg = ref.do(eagg, cpu_cache([cl[i]], [1], [vers[i]]), total=1, version=2)
        S.assert_bitwise(f"fedbuff subsets defer={defer}", {k: agg[k] for k in shapes}, eagg)
        bw = {k: v.to(DEV) for k, v in base.items() if v.is_floating_point()}
        ebw = {k: v.clone() for k, v in base.items() if v.is_floating_point()}
        opt.scale_add_agg_weights(bw, agg, 4)
        ref.scale_add_agg_weights(ebw, eagg, 4)
        S.assert_bitwise(f"fedbuff scale_add subsets defer={defer}", bw, ebw)
    # several subset arrivals queued in ONE deferred aggregate before its first read
    opt, ref = make_amd("fedbuff"), O.OracleFedBuff()
    agg = opt.do(None, cache_of([cl[0]], [1], [1]), total=1, version=2)
    eagg = ref.do(None, cpu_cache([cl[0]], [1], [1]), total=1, version=2)
    agg = opt.do(agg, cache_of(cl[1:], [1] * 3, vers[1:]), total=3, version=2)
    eagg = ref.do(eagg, cpu_cache(cl[1:], [1] * 3, vers[1:]), total=3, version=2)
    S.assert_bitwise("fedbuff queued subsets", {k: agg[k] for k in shapes}, eagg)
    with pytest.raises(KeyError):
        opt.do(agg, cache_of([{"zz": torch.ones(2)}], [1]), total=1, version=2)

    # FedAdam on fp32 keys (the kernel path; the SURVEY §8(c) contract is stated for fp32)
    fl = {k: v.float() for k, v in base.items() if v.is_floating_point()}
    fcl = [{k: v.float() for k, v in w.items() if k in fl} for w in cl]
    opt = make_amd("fedadam")
    ref = O.OracleFedOPT("fedadam")
    cur = {k: v.to(DEV) for k, v in fl.items()}
    ecur = {k: v.clone() for k, v in fl.items()}
    for r in range(3):
        cur = opt.do({k: v.clone() for k, v in cur.items()}, cache_of(fcl, counts), total=total)
        ecur = ref.do({k: v.clone() for k, v in ecur.items()}, cpu_cache(fcl, counts), total=total)
        if r == 0:
            S.assert_bitwise("fedadam subsets r0", cur, ecur)
        else:
            S.assert_close_fedopt(f"fedadam subsets r{r}", cur, ecur, elementwise=r == 1)


@pytest.mark.oracle
@pytest.mark.parametrize("sort", ["fedadam", "fedyogi"])
def test_fedopt_multichunk_multikey(sort):
    """FedOPT launches large enough for the 8-chunks-per-workgroup build (>= 16,384 fp32
    chunks): five keys (odd sizes, a 3-element and an empty key) in one launch, so a
    workgroup's chunks straddle keys and ragged key tails; slab and tensor placements equal
    each other bitwise (avg, m, v, cur), and the oracle within the §8(c) contract."""
    from flame_amd.slab import UpdateSlab
    O = _oracle()
    g = torch.Generator().manual_seed(23)
    shapes = {"a": (4_000_037,), "b": (3001, 4099), "c": (1_000_001,), "d": (3,), "e": (0,)}
    n, rounds = 6, 3
    w0 = {k: torch.randn(s, generator=g) for k, s in shapes.items()}
    data = [([{k: torch.randn(s, generator=g) * 1e-2 for k, s in shapes.items()} for _ in range(n)],
             torch.randint(1, 1000, (n,), generator=g).tolist()) for _ in range(rounds)]
    slab = UpdateSlab({k: torch.empty(s) for k, s in shapes.items()}, capacity=n, device=DEV)
    runs = {}
    for placement in ("slab", "tensors"):
        amd = make_amd(sort)
        wa = {k: v.to(DEV) for k, v in w0.items()}
        outs = []
        for cl, counts in data:
            c = S.SortedCache()
            for i in range(n):
                w = {k: v.to(DEV) for k, v in cl[i].items()}
                c[f"{i:02d}"] = S.TR(slab.put(w) if placement == "slab" else w, counts[i])
            wa = amd.do({k: v.clone() for k, v in wa.items()}, c, total=sum(counts))
            torch.cuda.synchronize()
            outs.append((S.to_cpu(dict(wa)), S.to_cpu(dict(amd.m_t)) if amd.m_t else None,
                         S.to_cpu(dict(amd.v_t)) if amd.v_t else None))
        runs[placement] = outs
    for r in range(rounds):
        for j, lbl in enumerate(("cur", "m", "v")):
            if runs["slab"][r][j] is not None:
                S.assert_bitwise(f"slab vs tensors r{r}/{lbl}", runs["slab"][r][j], runs["tensors"][r][j])
    ora = O.OracleFedOPT(sort)
    wo = {k: v.clone() for k, v in w0.items()}
    for r, (cl, counts) in enumerate(data):
        c = S.SortedCache()
        for i in range(n):
            c[f"{i:02d}"] = S.TR({k: v.clone() for k, v in cl[i].items()}, counts[i])
        wo = ora.do({k: v.clone() for k, v in wo.items()}, c, total=sum(counts))
        got = runs["slab"][r][0]
        if r == 0:
            S.assert_bitwise(f"{sort}/r0", got, wo)
        else:
            S.assert_close_fedopt(f"{sort}/r{r}/cur", got, wo, elementwise=r == 1)
            S.assert_close_fedopt(f"{sort}/r{r}/m", runs["slab"][r][1], ora.m_t, elementwise=r == 1)
