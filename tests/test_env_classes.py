"""The drop-ins' trainer-facing helper classes in both environments ("the
drop-in behaves differently depending on the environment and nothing tests that").

When flame is importable (a trainer or an aggregator running in flame's SDK), every
``.regularizer`` -- and FedGFT's server-side bias -- is flame's own class; otherwise it is
the restatement in flame_amd.  Both children run tests/env_probe.py; flame is made
importable the way tests/golden/make_golden.py does it (the reference tree + the
diskcache shim, no bytecode written).  The restatements must give the same values as
flame's classes on the same inputs.  Skipped where the reference tree is absent."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/lib/python"


def _probe(extra_path):
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1")
    env["PYTHONPATH"] = os.pathsep.join(p for p in (extra_path, env.get("PYTHONPATH", "")) if p)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "env_probe.py"), ROOT], env=env,
                         capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-3000:]
    return json.loads(out.stdout.strip().splitlines()[-1])


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree not present")
def test_regularizers_with_and_without_flame():
    alone = _probe("")
    shim = os.path.join(ROOT, "tests", "golden", "_shim")
    with_flame = _probe(os.pathsep.join((shim, REF)))
    for name in ("fedavg", "fedadam", "fedyogi", "fedadagrad", "fedbuff", "fedprox", "fedgft"):
        assert alone[name]["module"].startswith("flame_amd."), (name, alone[name])
        assert with_flame[name]["module"].startswith("flame."), (name, with_flame[name])
    for name in ("feddyn", "scaffold"):     # flame's own regularizers, or the no-op default without flame
        assert with_flame[name]["module"].startswith("flame."), (name, with_flame[name])
        assert alone[name]["module"].startswith("flame_amd."), (name, alone[name])
    assert alone["fedgft_bias_module"].startswith("flame_amd.")
    assert with_flame["fedgft_bias_module"].startswith("flame.")
    # same values from the restatements as from flame's classes
    assert alone["fedprox_term"] == with_flame["fedprox_term"]
    assert alone["fedgft_bias"] == with_flame["fedgft_bias"]
    assert alone["default_term"] == with_flame["default_term"]


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree not present")
def test_install_into_flame_provider():
    """``flame_amd.optimizers.install()`` with no argument re-registers every key of flame's own
    provider (optimizers.py:39-48, closed enum config.py:55-70), so a role's
    ``optimizer_provider.get(config.optimizer.sort, **config.optimizer.kwargs)``
    (syncfl/top_aggregator.py:97-99) on a job's optimizer block parsed by flame's pydantic
    ``Optimizer`` model (config.py:121-123, the type of ``Config.optimizer``) yields the drop-in with
    the job's kwargs."""
    shim = os.path.join(ROOT, "tests", "golden", "_shim")
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1")
    env["PYTHONPATH"] = os.pathsep.join(p for p in (shim, REF, env.get("PYTHONPATH", "")) if p)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "install_probe.py"), ROOT], env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    keys = {"fedavg", "fedadam", "fedyogi", "fedadagrad", "fedbuff", "fedprox", "feddyn", "scaffold", "fedgft"}
    assert set(out["before"]) == keys and set(out["after"]) == keys
    for k in keys:
        assert out["before"][k].startswith("flame.optimizer."), (k, out["before"][k])
        assert out["after"][k]["cls"].startswith("flame_amd.optimizer."), (k, out["after"][k])
        assert out["after"][k]["same_as_drop_in"], k
    assert out["returned_flame_provider"] is True
    assert out["unknown_key"] == "ValueError:fedsgd"
    c = out["config"]
    assert c["fedyogi"]["cls"] == "flame_amd.optimizer.fedyogi.FedYogi" and c["fedyogi"]["sort"] == "fedyogi"
    assert c["fedyogi"]["hyper"] == [0.85, 0.995, 0.02, 0.002]
    assert c["fedadam"]["cls"] == "flame_amd.optimizer.fedadam.FedAdam"
    assert c["fedadam"]["hyper"] == [0.9, 0.99, 0.01, 0.001]
    assert c["fedbuff"]["cls"] == "flame_amd.optimizer.fedbuff.FedBuff"
    assert c["fedavg_default"]["cls"] == "flame_amd.optimizer.fedavg.FedAvg"
    assert c["fedavg_default"]["sort"] == "fedavg"
    for name in c:      # flame's own regularizer class when flame is importable; empty round -> None
        assert c[name]["regularizer"].startswith("flame."), (name, c[name])
        assert c[name]["empty_do"] == "None", (name, c[name])
    assert out["bad_sort"] == "ValidationError"
