"""Guard: every host-side launch branch of the C ABI is reached by a passing oracle test.

Runs last in the GPU session (file order).  tests/conftest.py attributes every GPU
test's launches to the branches of flame_launch_branch_count (one per kernel
instantiation a launch entry point can pick: dtype x variant x residency x store-group
mode x metadata path) and credits them only to tests that are marked ``oracle``, consulted
the CPU oracle or a golden fixture while they ran, and passed.  A branch reached only by
HIP-vs-HIP self-comparisons would be a kernel the product can run with no oracle evidence.
The branch -> tests map (credited and other) is written to
gpurun_out/launch_branches.json when that directory exists.
"""
import json
import os

import pytest

import conftest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GPU_FILES = sorted(f for f in os.listdir(HERE) if f.startswith("test_gpu_") and f.endswith(".py")
                   and f != os.path.basename(__file__))


def test_every_launch_branch_reached_by_an_oracle_test():
    missing_files = [f for f in GPU_FILES if f not in conftest.COLLECTED_FILES]
    if missing_files:
        pytest.skip(f"partial GPU session (not collected: {', '.join(missing_files)})")
    from flame_amd import _native
    names = list(_native.launch_branch_counts())
    hits = {n: sorted(set(conftest.BRANCH_HITS.get(n, []))) for n in names}
    other = {n: sorted(set(conftest.BRANCH_OTHER.get(n, []))) for n in names}
    out = os.path.join(os.path.dirname(HERE), "gpurun_out")
    if os.path.isdir(out):
        with open(os.path.join(out, "launch_branches.json"), "w") as f:
            json.dump({"branches": len(names), "credit": "passed oracle-marked tests that consulted a checker",
                       "oracle_hits": {n: len(t) for n, t in hits.items()},
                       "other_hits": {n: len(t) for n, t in other.items()},
                       "oracle_tests": hits, "other_tests": other}, f, indent=1)
    unreached = [n for n, t in hits.items() if not t]
    assert not unreached, (f"{len(unreached)} of {len(names)} launch branches reached by no passing oracle test "
                           f"(self-comparisons do not count): {unreached}")
