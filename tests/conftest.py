import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests", "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")


@pytest.fixture
def golden():
    from fixture_io import Fixture

    def load(name):
        return Fixture(os.path.join(GOLDEN, name))
    return load


# ------------------------------------------------------------------ launch-branch bookkeeping
# Every GPU test's native launches are attributed to the C ABI's launch branches
# (flame_launch_branch_count before/after the test); tests/test_gpu_zz_launch_branches.py
# then checks that the session's oracle tests reached every branch.
BRANCH_HITS = {}          # branch name -> [test node ids]
COLLECTED_FILES = set()   # basenames of the test files this session collected


def pytest_collection_modifyitems(session, config, items):
    for it in items:
        COLLECTED_FILES.add(os.path.basename(str(it.fspath)))


@pytest.fixture(autouse=True)
def _launch_branches(request):
    if request.node.get_closest_marker("gpu") is None:
        yield
        return
    try:
        from flame_amd import _native
        before = _native.launch_branch_counts()
    except Exception:  # noqa: BLE001 - no library: the test itself fails loudly
        yield
        return
    yield
    after = _native.launch_branch_counts()
    for name, n in after.items():
        BRANCH_HITS.setdefault(name, [])
        if n > before.get(name, 0):
            BRANCH_HITS[name].append(request.node.nodeid)
