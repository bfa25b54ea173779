"""Maximum sizes: one state_dict key of more than 2^31 elements (8.6 GB of fp32, every byte
offset past 4 GiB and every element index past 2^31) through the drop-ins -- FedAvg (client
tensors and the tiled slab, whose insert is one flame_slab_write launch of 2M tiles),
FedBuff's fused scale_add + delta (the hierarchy kernel with one middle) and FedAdam's
fused adaptive round -- checked against the oracle at the index boundaries (2^30, 2^31, the
chunk seams, the ragged tail) and 20,000 random indices.  Inputs come from the counter
generator on the device; only the sampled elements travel to the host."""
import numpy as np
import pytest
import torch

import scenarios as S

pytestmark = [pytest.mark.gpu, pytest.mark.oracle]

DEV = "cuda:0"
P = (1 << 31) + 4099           # a ragged tail after the 2^31st element


def _need(gb):
    free, _ = torch.cuda.mem_get_info()
    if free < gb * 1e9:
        pytest.skip(f"needs {gb} GB of HBM, {free / 1e9:.1f} GB free")


def _synth(seed, stream, sigma):
    from flame_amd import engine
    t = torch.empty(P, device=DEV)
    engine.synth_fill_(t, seed, stream, 0, sigma)
    return t


def _index():
    edges = []
    for b in (0, 1 << 30, (1 << 31) - 2048, 1 << 31, P - 4099, P - 2048):
        edges += list(range(max(0, b - 3), min(P, b + 3)))
    edges += [1023, 1024, 1025, 2047, 2048, P - 1]
    rand = np.random.default_rng(0).integers(0, P, 20_000)
    return torch.from_numpy(np.unique(np.concatenate([np.array(edges), rand])).astype(np.int64))


def _at(t, idx):
    return t.index_select(0, idx.to(t.device)).cpu()


def _free():
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def _make(sort, **kw):
    from flame_amd.optimizers import optimizer_provider
    return optimizer_provider.get(sort, **kw)


@pytest.mark.parametrize("placement", ["tensors", "slab"])
def test_fedavg_one_key_past_2_31_elements(placement):
    from oracle import oracle as O
    from flame_amd.slab import UpdateSlab
    n, counts = 3, [3, 5, 11]
    _need((n + 2) * P * 4 / 1e9 + 2)
    idx = _index()
    base = _synth(9, 0, 1.0)
    ups = [_synth(9, 1 + i, 1e-2) for i in range(n)]
    b_s, u_s = _at(base, idx), [_at(u, idx) for u in ups]
    if placement == "slab":
        slab = UpdateSlab({"w": torch.empty(P, device="meta")}, capacity=n, device=DEV)
        ws = [slab.put({"w": u}) for u in ups]
        del ups
        _free()
        for i, w in enumerate(ws):         # the one-launch insert of an 8.6 GB key, read back
            assert torch.equal(_at(slab.read(w.slot, "w"), idx), u_s[i])
    else:
        ws = [{"w": u} for u in ups]
    cache, ocache = S.SortedCache(), S.SortedCache()
    for i in range(n):
        cache[f"{i}"] = S.TR(ws[i], counts[i])
        ocache[f"{i}"] = S.TR({"w": u_s[i]}, counts[i])
    out = _make("fedavg").do({"w": base}, cache, total=sum(counts))
    exp = O.OracleFedAvg().do({"w": b_s.clone()}, ocache, total=sum(counts))
    S.assert_bitwise(f"fedavg/{placement}", {"w": _at(out["w"], idx)}, exp)
    del out, base, ws, cache
    _free()


def test_fedbuff_fused_scale_add_past_2_31_elements():
    """Two queued arrivals reduced straight into the model with the middle's upload delta
    (one flame_hier_fedbuff launch) == the oracle's do(), do(), scale_add + delta."""
    from oracle import oracle as O
    _need(6 * P * 4 / 1e9 + 2)
    idx = _index()
    w = _synth(10, 0, 1.0)
    ups = [_synth(10, 1 + i, 1e-2) for i in range(2)]
    w_s, u_s = _at(w, idx), [_at(u, idx) for u in ups]
    vers, rnd, goal = [7, 5], 7, 2
    opt, agg = _make("fedbuff"), None
    ora, oagg = O.OracleFedBuff(), None
    for i in range(2):
        c, oc = S.SortedCache(), S.SortedCache()
        c["e"] = S.TR({"w": ups[i]}, 1, vers[i])
        oc["e"] = S.TR({"w": u_s[i]}, 1, vers[i])
        agg = opt.do(agg, c, total=1, version=rnd)
        oagg = ora.do(oagg, oc, total=1, version=rnd)
    _, delta = opt.scale_add_agg_weights_with_delta({"w": w}, agg, goal)
    ow = w_s.clone()
    od = O.scale_add_tensor(ow, oagg["w"], goal, want_delta=True)
    S.assert_bitwise("fedbuff/w", {"w": _at(w, idx)}, {"w": ow})
    S.assert_bitwise("fedbuff/delta", {"w": _at(delta["w"], idx)}, {"w": od})
    del w, ups, agg, delta
    _free()


def test_fedadam_past_2_31_elements():
    """Round 1 (passthrough) and an adaptive round (the fused reduce + adapt kernel, zero
    state) against OracleFedOPT at the sampled elements: the average bitwise, cur / m / v
    within the SURVEY §8(c) contract."""
    from oracle import oracle as O
    _need(10 * P * 4 / 1e9 + 2)
    idx = _index()
    opt, ora = _make("fedadam"), O.OracleFedOPT("fedadam")
    cur = _synth(11, 0, 1.0)
    ocur = _at(cur, idx)
    counts = [4, 9]
    for r in range(2):
        ups = [_synth(11, 10 * (r + 1) + i, 1e-2) for i in range(2)]
        c, oc = S.SortedCache(), S.SortedCache()
        for i in range(2):
            c[f"{i}"] = S.TR({"w": ups[i]}, counts[i])
            oc[f"{i}"] = S.TR({"w": _at(ups[i], idx)}, counts[i])
        # the caller's do(deepcopy(self.weights), ...) (syncfl/top_aggregator.py:161-166)
        cur = opt.do({"w": cur.clone()}, c, total=sum(counts))["w"]
        ocur = ora.do({"w": ocur.clone()}, oc, total=sum(counts))["w"]
        del ups, c
        _free()
        S.assert_bitwise(f"fedadam/r{r}/avg", {"w": _at(opt.agg_weights["w"], idx)}, ora.agg_weights)
        if r == 0:
            S.assert_bitwise("fedadam/r0/cur", {"w": _at(cur, idx)}, {"w": ocur})
        else:
            S.assert_close_fedopt("fedadam/r1/cur", {"w": _at(cur, idx)}, {"w": ocur})
            S.assert_close_fedopt("fedadam/r1/m", {"w": _at(opt.m_t["w"], idx)}, ora.m_t)
            S.assert_close_fedopt("fedadam/r1/v", {"w": _at(opt.v_t["w"], idx)}, ora.v_t)
    del cur, opt
    _free()


@pytest.mark.parametrize("placement", ["slab", "tensors"])
def test_bf16_hierarchy_round_past_2_31_elements(placement):
    """Config 5's kernel (flame_hier_fedbuff, middles + top in one pass) on one bf16 key of
    2^31 + 4099 elements: 2 middles x 2 arrivals, middle weights, deltas, top aggregate and
    top weights against the oracle's op sequence at the sampled elements, bitwise."""
    from oracle import oracle as O
    from flame_amd import engine
    from flame_amd.optimizer.fedbuff import hierarchy_round
    from flame_amd.slab import UpdateSlab
    M, C, rnd, goals, mid_ver, top_goal = 2, 2, 9, [2, 3], [9, 8], 2
    vers = [[9, 7], [8, 9]]
    _need(12 * P * 2 / 1e9 + 2)
    idx = _index()

    def bf(seed, stream, sigma):
        t = torch.empty(P, dtype=torch.bfloat16, device=DEV)
        engine.synth_fill_(t, seed, stream, 0, sigma)
        return t
    ups = [[bf(12, 1 + m * C + t, 1e-2) for t in range(C)] for m in range(M)]
    mids = [bf(12, 100 + m, 1.0) for m in range(M)]
    top_w = bf(12, 200, 1.0)
    u_s = [[_at(u, idx) for u in row] for row in ups]
    mid_s, top_s = [_at(x, idx) for x in mids], _at(top_w, idx)
    slab = UpdateSlab({"w": torch.empty(P, dtype=torch.bfloat16, device="meta")}, capacity=M * C, device=DEV) \
        if placement == "slab" else None
    aggs = []
    for m in range(M):
        opt, agg = _make("fedbuff"), None
        for t in range(C):
            c = S.SortedCache()
            c["a"] = S.TR(slab.put({"w": ups[m][t]}) if slab is not None else {"w": ups[m][t]}, 1, vers[m][t])
            agg = opt.do(agg, c, total=1, version=rnd)
        aggs.append(agg)
    if slab is not None:
        del ups
        _free()
    mids_w = [{"w": x} for x in mids]
    top_agg, deltas = hierarchy_round([(mids_w[m], aggs[m], goals[m], mid_ver[m]) for m in range(M)], None,
                                      version=rnd, top_weights={"w": top_w}, top_goal=top_goal, with_delta=True)
    top_o, top_agg_o = O.OracleFedBuff(), None
    for m in range(M):
        mo, agg_o = O.OracleFedBuff(), None
        for t in range(C):
            c = S.SortedCache()
            c["a"] = S.TR({"w": u_s[m][t]}, 1, vers[m][t])
            agg_o = mo.do(agg_o, c, total=1, version=rnd)
        w = {"w": mid_s[m].clone()}
        d = {"w": O.scale_add_tensor(w["w"], agg_o["w"], goals[m], want_delta=True)}
        S.assert_bitwise(f"hier/{placement}/mid{m}", {"w": _at(mids[m], idx)}, w)
        S.assert_bitwise(f"hier/{placement}/delta{m}", {"w": _at(deltas[m]["w"], idx)}, d)
        c = S.SortedCache()
        c["d"] = S.TR(d, 1, mid_ver[m])
        top_agg_o = top_o.do(top_agg_o, c, total=1, version=rnd)
    S.assert_bitwise(f"hier/{placement}/top agg", {"w": _at(top_agg["w"], idx)}, top_agg_o)
    tw = {"w": top_s.clone()}
    top_o.scale_add_agg_weights(tw, top_agg_o, top_goal)
    S.assert_bitwise(f"hier/{placement}/top w", {"w": _at(top_w, idx)}, tw)
    del mids, top_w, aggs, deltas, top_agg
    _free()
