"""Pin the CPU oracle against golden vectors produced by the REAL reference.

Bitwise for FedAvg / FedBuff (every dtype the fixtures hold); FedOPT within the
SURVEY §8(c) tolerance (torch-CPU fp32 sqrt is not correctly rounded).
"""
import pytest

import scenarios as S
from oracle import oracle as O


def make_oracle(sort, **kw):
    if sort == "fedavg":
        return O.OracleFedAvg()
    if sort == "fedbuff":
        return O.OracleFedBuff()
    return O.OracleFedOPT(sort, **kw)


@pytest.mark.parametrize("name,driver", S.BITWISE_FIXTURES, ids=[n for n, _ in S.BITWISE_FIXTURES])
def test_oracle_bitwise(golden, name, driver):
    for label, got, exp in driver(golden(name), make_oracle, "cpu"):
        S.assert_bitwise(f"{name}:{label}", got, exp)


@pytest.mark.parametrize("name", S.FEDOPT_FIXTURES)
def test_oracle_fedopt(golden, name):
    for label, got, exp in S.run_fedopt(golden(name), make_oracle, "cpu"):
        if label in ("r0/cur", "r0/avg", "r1/avg"):
            # before any adaptive step everything is FedAvg arithmetic: bitwise
            S.assert_bitwise(f"{name}:{label}", got, exp)
        else:
            S.assert_close_fedopt(f"{name}:{label}", got, exp)


def test_oracle_hier(golden):
    for label, got, exp in S.run_hier(golden("hier_fedbuff_small.npz"), make_oracle, "cpu", S.delta_torch):
        S.assert_bitwise(label, got, exp)


def test_oracle_synth_matches_numpy():
    import numpy as np
    from flame_amd import synth
    for seed, stream, start, n in [(0, 0, 0, 1000), (2, 1023, 24_999_000, 1000), (4, 4095, 7, 3)]:
        a = O.synth_f32(seed, stream, start, n, synth.scale_for_sigma(0.01))
        b = synth.synth_f32(seed, stream, np.arange(start, start + n), 0.01)
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
