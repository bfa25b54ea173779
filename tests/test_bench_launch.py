"""bench.py --gpus N means N ranks, whatever starts it: the launch decision
is made before anything touches the GPU, a bare ``--gpus N`` (N > 1) starts N ranks under
torch.distributed.run in child processes, and a launcher whose world disagrees with --gpus is
an error, not a mislabelled line.  CPU only: the spawn is intercepted."""
import io
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


@pytest.mark.parametrize("gpus,env,want", [
    (1, {}, ("run", None)),
    (2, {}, ("spawn", 2)),
    (8, {}, ("spawn", 8)),
    (8, {"WORLD_SIZE": "8", "RANK": "3"}, ("run", None)),
    (1, {"WORLD_SIZE": "1", "RANK": "0"}, ("run", None)),
    (2, {"RANK": "0"}, ("run", None)),
])
def test_launch_plan(gpus, env, want):
    assert bench.launch_plan(gpus, env) == want


@pytest.mark.parametrize("gpus,ws", [(8, "4"), (1, "2"), (2, "1")])
def test_launch_plan_world_mismatch_is_an_error(gpus, ws):
    what, msg = bench.launch_plan(gpus, {"WORLD_SIZE": ws, "RANK": "0"})
    assert what == "error" and f"--gpus {gpus}" in msg and f"WORLD_SIZE is {ws}" in msg


def test_launch_plan_rejects_zero():
    assert bench.launch_plan(0, {})[0] == "error"


def _no_gpu(*a, **k):
    raise AssertionError("the launching parent touched the GPU")


def test_main_spawns_before_touching_the_gpu(monkeypatch):
    """``bench.py --gpus 4`` with no launcher env: main() hands off to spawn_ranks before
    setup_dist / torch.cuda / the native library, and exits with the ranks' exit code."""
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setattr(torch.cuda, "set_device", _no_gpu)
    monkeypatch.setattr(torch.cuda, "is_available", _no_gpu)
    monkeypatch.setattr(bench, "setup_dist", _no_gpu)
    seen = {}

    def fake_spawn(n, argv):
        seen["n"], seen["argv"] = n, argv
        return 7
    monkeypatch.setattr(bench, "spawn_ranks", fake_spawn)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "3", "--warmup", "1"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 7
    assert seen == {"n": 4, "argv": ["--gpus", "4", "--steps", "3", "--warmup", "1"]}


def test_main_mismatch_exits_nonzero(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "8")
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setattr(bench, "setup_dist", _no_gpu)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert isinstance(e.value.code, str) and "WORLD_SIZE is 8" in e.value.code


def test_spawn_ranks_command_and_relay(monkeypatch, capsys):
    """The child command is torch.distributed.run with N ranks on 127.0.0.1 running this very
    script with the same arguments; rank 0's JSON line is relayed to stdout; the launcher's
    exit code is returned."""
    import subprocess
    got = {}

    class P:
        def __init__(self, cmd, env, **kw):
            got["cmd"], got["env"] = cmd, env
            self.stdout = io.StringIO('{"metric": "m", "n_gpus": 3}\n')

        def wait(self):
            return 0
    monkeypatch.setattr(subprocess, "Popen", P)
    rc = bench.spawn_ranks(3, ["--gpus", "3", "--steps", "2"])
    cmd = got["cmd"]
    assert rc == 0
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=3" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-5:] == [os.path.join(ROOT, "bench.py"), "--gpus", "3", "--steps", "2"]
    assert "torch.distributed.run" in got["env"]["FLAME_BENCH_LAUNCHER"]
    assert capsys.readouterr().out == '{"metric": "m", "n_gpus": 3}\n'
