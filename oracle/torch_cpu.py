"""Op-for-op torch-CPU restatement of the reference aggregation loops.

TEST / BASELINE INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg and tests).
It is the reference's own arithmetic and op sequence, not a new algorithm:

  fedavg_round      lib/python/flame/optimizer/fedavg.py:79-104
                    for k in cache.iterkeys(): rate = count/total;
                        tmp = v * rate; tmp = tmp.to(v.dtype) if needed; agg[k] += tmp
  fedbuff_step      lib/python/flame/optimizer/fedbuff.py:94-96,136-157
  fedbuff_scale_add lib/python/flame/optimizer/fedbuff.py:122-127
  fedopt_adapt      lib/python/flame/optimizer/fedopt.py:102-129 + the _delta_v variants
                    (fedadam.py:33-35, fedyogi.py:34-36, fedadagrad.py:33-35)

Being the same torch CPU kernels, it runs at the reference's speed minus the
diskcache disk round trip (favourable to the reference) and is
bit-identical to it (tests/test_oracle_golden.py::test_torch_cpu_matches_golden).
"""
import math

import torch

try:
    from . import consult
except ImportError:  # loaded as a top-level module
    import consult


def fedavg_round(agg_weights, updates, counts, total):
    """agg_weights[k] += (v * count/total) for each update in order (in place)."""
    consult.note()
    for w, c in zip(updates, counts):
        rate = c / total
        for k, v in w.items():
            tmp = v * rate
            tmp = tmp.to(dtype=v.dtype) if tmp.dtype != v.dtype else tmp
            agg_weights[k] += tmp
    return agg_weights


def fedbuff_step(agg, weights, version, tres_version):
    consult.note()
    rate = 1 / math.sqrt(1 + version - tres_version)
    if agg is None:
        agg = {}
        for k, v in weights.items():
            tmp = v * rate
            agg[k] = tmp.to(dtype=v.dtype) if tmp.dtype != v.dtype else tmp
        return agg
    for k, v in weights.items():
        tmp = v * rate
        tmp = tmp.to(dtype=v.dtype) if tmp.dtype != v.dtype else tmp
        agg[k] += tmp
    return agg


def fedbuff_scale_add(base_weights, agg_goal_weights, agg_goal):
    consult.note()
    for k in base_weights.keys():
        base_weights[k] += agg_goal_weights[k] / agg_goal
    return base_weights


def fedopt_adapt(sort, avg, cur, m_t, v_t, beta_1, beta_2, eta, tau):
    """One adaptive step per key; m_t / v_t dicts are updated (None entries start at zeros)."""
    consult.note()
    new = {}
    for k in cur.keys():
        d = avg[k] - cur[k]
        m = m_t.get(k)
        m = beta_1 * (m if m is not None else d.new_zeros(d.shape)) + (1 - beta_1) * d
        v = v_t.get(k)
        v = v if v is not None else d.new_zeros(d.shape)
        if sort == "fedadam":
            v = beta_2 * v + (1 - beta_2) * d**2
        elif sort == "fedyogi":
            v = v - (1 - beta_2) * d**2 * torch.sign(v - d**2)
        else:
            v = v + d**2
        m_t[k], v_t[k] = m, v
        new[k] = cur[k] + eta * m_t[k] / (torch.sqrt(v_t[k]) + tau)
    return new
