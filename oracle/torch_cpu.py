"""Op-for-op torch-CPU restatement of the reference aggregation loops.

TEST / BASELINE INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg and tests).
It is the reference's own arithmetic and op sequence, not a new algorithm:

  fedavg_round      lib/python/flame/optimizer/fedavg.py:79-104
                    for k in cache.iterkeys(): rate = count/total;
                        tmp = v * rate; tmp = tmp.to(v.dtype) if needed; agg[k] += tmp
  fedbuff_step      lib/python/flame/optimizer/fedbuff.py:94-96,136-157

Being the same torch CPU kernels, it runs at the reference's speed minus the
diskcache disk round trip (favourable to the reference) and is
bit-identical to it (tests/test_oracle_golden.py::test_torch_cpu_matches_golden).
"""
import math


def fedavg_round(agg_weights, updates, counts, total):
    """agg_weights[k] += (v * count/total) for each update in order (in place)."""
    for w, c in zip(updates, counts):
        rate = c / total
        for k, v in w.items():
            tmp = v * rate
            tmp = tmp.to(dtype=v.dtype) if tmp.dtype != v.dtype else tmp
            agg_weights[k] += tmp
    return agg_weights


def fedbuff_step(agg, weights, version, tres_version):
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
