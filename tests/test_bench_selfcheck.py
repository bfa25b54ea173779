"""bench.py's N>1 self-check, pinned on the CPU: its host restatements of the sharded lines
(FedAvg / FedOPT rounds, config 5's async and sync hierarchy in bf16) equal the oracle's
do() restatements on the same counter-generated inputs, bitwise; the sampled indices
cover every wave, every rank boundary and the replicated tails."""

import numpy as np
import torch

import bench
import scenarios as S
from flame_amd import shard, synth


def _oracle():
    from oracle import oracle as O
    return O


def _t(x, dtype=torch.float32):
    t = torch.from_numpy(np.asarray(x, dtype=np.float32).copy())
    return t.to(dtype) if dtype != torch.float32 else t


def test_sample_indices_cover_waves_boundaries_and_tails():
    plan = shard.ShardPlan({"model": torch.empty(3 * 8 * 2048 * 5 + 333, device="meta")}, 8, 3)
    idx = bench.sample_indices(plan, "model", per_wave=16, seed=1)
    assert idx.min() >= 0 and idx.max() < plan.numel["model"]
    for s in plan.subs:
        inside = np.count_nonzero((idx >= s.g0) & (idx < s.g1))
        assert inside >= (16 if not s.tail else min(16, s.g1 - s.g0)), s
        if not s.tail:
            per = (s.g1 - s.g0) // 8
            for r in range(8):
                assert s.g0 + r * per in idx and s.g0 + (r + 1) * per - 1 in idx


def test_host_fedavg_rounds_equals_oracle():
    O = _oracle()
    seed, n, P, rounds = 7, 9, 257, 3
    idx = np.arange(P)
    counts = synth.counts(seed, n)
    total = int(counts.sum())
    base = {"m": _t(synth.synth_f32(seed, 0, idx, 1.0))}
    cl = [_t(synth.synth_f32(seed, 1 + i, idx, 1e-2)) for i in range(n)]
    for _ in range(rounds):
        c = S.SortedCache()
        for i in range(n):
            c[f"{i:05d}"] = S.TR({"m": cl[i]}, int(counts[i]))
        O.OracleFedAvg().do(base, c, total=total)
    got = bench.host_fedavg_rounds(seed, counts, idx, rounds)
    assert np.array_equal(got.view(np.uint32), base["m"].numpy().view(np.uint32))


def test_host_fedopt_rounds_equals_oracle():
    O = _oracle()
    seed, n, P, rounds = 3, 6, 301, 4
    idx = np.arange(P)
    counts = synth.counts(seed, n)
    total = int(counts.sum())
    cl = [_t(synth.synth_f32(seed, 1 + i, idx, 1e-2)) for i in range(n)]
    for sort in ("fedadam", "fedyogi", "fedadagrad"):
        ora = O.OracleFedOPT(sort)
        cur = {"m": _t(synth.synth_f32(seed, 0, idx, 1.0))}
        for _ in range(rounds):
            c = S.SortedCache()
            for i in range(n):
                c[f"{i:05d}"] = S.TR({"m": cl[i]}, int(counts[i]))
            cur = ora.do({"m": cur["m"].clone()}, c, total=total)
        got = bench.host_fedopt_rounds(sort, O.fedopt_scalars(0.9, 0.99, 1e-2, 1e-3), seed, counts, idx, rounds)
        assert np.array_equal(got.view(np.uint32), cur["m"].numpy().view(np.uint32)), sort


def _oracle_hier_round(O, gw, mids, arr, stale, cnt, M, C, rnd, fetched, sync, shared):
    """The roles' separate calls on the oracle (bf16 tensors)."""
    if sync:
        totals = [int(cnt[m * C:(m + 1) * C].sum()) for m in range(M)]
        top_total = sum(totals)
        top_c = S.SortedCache()
        for m in range(M):
            w = shared if fetched else mids[m]
            c = S.SortedCache()
            for t in range(C):
                c[f"{m * C + t:05d}"] = S.TR({"m": arr[m * C + t]}, int(cnt[m * C + t]))
            new = O.OracleFedAvg().do({"m": w.clone()}, c, total=totals[m])["m"]
            top_c[f"mid{m:03d}"] = S.TR({"m": new - w}, totals[m])
            if not fetched:
                mids[m] = new
        O.OracleFedAvg().do({"m": gw}, top_c, total=top_total)
        return gw
    top = O.OracleFedBuff()
    tagg = None
    for m in range(M):
        w = shared if fetched else mids[m]
        fb = O.OracleFedBuff()
        agg = None
        for t in range(C):
            c = S.SortedCache()
            c["a"] = S.TR({"m": arr[m * C + t]}, 1, rnd - stale[m * C + t])
            agg = fb.do(agg, c, total=1, version=rnd)
        nw = w.clone()
        d = O.scale_add_tensor(nw, agg["m"], C, want_delta=True)
        if not fetched:
            mids[m] = nw
        c = S.SortedCache()
        c["mid"] = S.TR({"m": d}, C, rnd - m % 2)
        tagg = top.do(tagg, c, total=C, version=rnd)
    top.scale_add_agg_weights({"m": gw}, tagg, M)
    return gw


def test_host_hier_rounds_equals_oracle():
    O = _oracle()
    seed, M, C, P, rounds, rnd = 11, 3, 5, 199, 2, 10
    idx = np.arange(P)
    cnt = synth.counts(seed, M * C)
    stale = [int(x) % 4 for x in cnt]
    arr = [_t(synth.synth_f32(seed, 1 + i, idx, 1e-2), torch.bfloat16) for i in range(M * C)]
    for sync in (False, True):
        for fetched in (False, True):
            gw = _t(synth.synth_f32(seed, 0, idx, 1.0), torch.bfloat16)
            shared = gw.clone()
            mids = [gw.clone() for _ in range(M)]
            for _ in range(rounds):
                gw = _oracle_hier_round(O, gw, mids, arr, stale, cnt, M, C, rnd, fetched, sync, shared)
            got = bench.host_hier_rounds(seed, M, C, idx, rounds, rnd, fetched, sync)
            exp = synth.f32_to_bf16_bits(gw.float().numpy())
            assert np.array_equal(synth.f32_to_bf16_bits(got), exp), (sync, fetched)
