"""bench.py's eager lines at 16-bit dtypes: argument routing and the CPU baseline leg (the
reference's eager round op sequence in the model's dtype).  CPU only."""
import os
import subprocess
import sys

import torch

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_dtype_is_refused_outside_the_eager_workloads():
    for argv in (["--dtype", "bf16"], ["--dtype", "f16", "--workload", "fedadam"],
                 ["--dtype", "bf16", "--e2e", "--workload", "fedadam_eager"]):
        r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *argv], capture_output=True, text=True,
                           timeout=120, env=dict(os.environ, CUDA_VISIBLE_DEVICES=""))
        assert r.returncode != 0
        assert "fed*_eager workloads only" in r.stderr, r.stderr[-400:]


def _rows(n, P, dtype):
    g = torch.Generator().manual_seed(7)
    return [(torch.randn(P, generator=g) * 1e-2).to(dtype) for _ in range(n)]


def test_cpu_baseline_eager_runs_the_reference_round_in_the_dtype():
    n, P = 6, 4096
    for dtype in (torch.float32, torch.bfloat16, torch.float16):
        rows = _rows(n, P, dtype)
        base0 = torch.linspace(-1, 1, P).to(dtype)
        counts = [3, 5, 2, 7, 1, 4]
        for sort in ("fedavg", "fedadam", "fedyogi", "fedadagrad"):
            res = bench.cpu_baseline_eager(sort, lambda i: rows[i], n, P, base0, counts, 4, 1)
            assert res["value"] > 0 and res["kind"] == "port" and res["cores"] >= 1
            assert f"first 4 of the {n} arrivals x {P} {str(dtype).replace('torch.', '')}" in res["sample"]
            assert ("fedopt.py:102-129" in res["sample"]) == (sort != "fedavg")

