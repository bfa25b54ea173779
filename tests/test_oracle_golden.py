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
    if sort == "feddyn":
        return O.OracleFedDyn(**kw)
    if sort == "scaffold":
        return O.OracleScaffold(**kw)
    if sort == "fedgft":
        return O.OracleFedGFT(**kw)
    return O.OracleFedOPT(sort, **kw)


@pytest.mark.parametrize("name,driver", S.BITWISE_FIXTURES, ids=[n for n, _ in S.BITWISE_FIXTURES])
def test_oracle_bitwise(golden, name, driver):
    for label, got, exp in driver(golden(name), make_oracle, "cpu"):
        S.assert_bitwise(f"{name}:{label}", got, exp)


def test_oracle_nonfinite(golden):
    """nonfinite.npz (the reference's FedAvg / FedBuff over a diverged trainer's updates):
    NaN and +-inf where the reference puts them, every other element bitwise."""
    labels = []
    for label, got, exp in S.run_nonfinite(golden("nonfinite.npz"), make_oracle, "cpu"):
        S.assert_same_nonfinite(f"nonfinite:{label}", got, exp)
        labels.append(label)
    assert len(labels) == 12


@pytest.mark.parametrize("name", S.FEDOPT_FIXTURES)
def test_oracle_fedopt(golden, name):
    for label, got, exp in S.run_fedopt(golden(name), make_oracle, "cpu"):
        rnd = int(label.split("/")[0][1:])
        if label in ("r0/cur", "r0/avg", "r1/avg"):
            # before any adaptive step everything is FedAvg arithmetic: bitwise
            S.assert_bitwise(f"{name}:{label}", got, exp)
        else:
            # rounds >= 2 start from state that already differs by sqrt ulps: rel-L2 contract
            S.assert_close_fedopt(f"{name}:{label}", got, exp, elementwise=rnd <= 1)


@pytest.mark.parametrize("name", S.FEDOPT_FIXTURES)
def test_oracle_fedopt_single_round_elementwise(golden, name):
    fx = golden(name)
    m = fx.meta
    for r, clients, counts, state, exp in S.fedopt_identical_state_rounds(fx, "cpu"):
        opt = O.OracleFedOPT(m["sort"], beta_1=m["beta_1"], beta_2=m["beta_2"], eta=m["eta"], tau=m["tau"])
        opt.current_weights = state["cur"]
        opt.m_t, opt.v_t = state["m"], state["v"]
        cache = S.SortedCache()
        for i, (w, c) in enumerate(zip(clients, counts)):
            cache[f"{i:03d}"] = S.TR(w, c)
        out = opt.do({k: v.clone() for k, v in state["cur"].items()}, cache, total=sum(counts))
        S.assert_bitwise(f"{name}:r{r}/avg", opt.agg_weights, exp["avg"])
        for key in ("cur", "m", "v"):
            got = out if key == "cur" else getattr(opt, key + "_t")
            S.assert_close_fedopt(f"{name}:r{r}/{key}", got, exp[key])


@pytest.mark.parametrize("name", S.HIER_FIXTURES)
def test_oracle_hier(golden, name):
    for label, got, exp in S.run_hier(golden(name), make_oracle, "cpu", S.delta_torch):
        S.assert_bitwise(f"{name}:{label}", got, exp)


def test_oracle_synth_matches_numpy():
    import numpy as np
    from flame_amd import synth
    for seed, stream, start, n in [(0, 0, 0, 1000), (2, 1023, 24_999_000, 1000), (4, 4095, 7, 3)]:
        a = O.synth_f32(seed, stream, start, n, synth.scale_for_sigma(0.01))
        b = synth.synth_f32(seed, stream, np.arange(start, start + n), 0.01)
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.mark.parametrize("name", S.FEDOPT_EAGER_FIXTURES)
def test_oracle_fedopt_eager(golden, name):
    """FedOPT under the eager caller (current aliases base after the round-1 passthrough)."""
    from oracle import oracle as O

    def make(sort, **kw):
        return O.OracleFedOPT(sort, **kw)
    S.check_fedopt_eager(S.run_fedopt_eager(golden(name), make, "cpu"))
