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
