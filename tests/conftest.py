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
    config.addinivalue_line("markers", "oracle: compares the HIP path with the CPU oracle or a golden fixture "
                                       "(credits launch branches; see _launch_branches)")


@pytest.fixture
def golden():
    from fixture_io import Fixture

    def load(name):
        return Fixture(os.path.join(GOLDEN, name))
    return load


# ------------------------------------------------------------------ launch-branch bookkeeping
# Every GPU test's native launches are attributed to the C ABI's launch branches
# (flame_launch_branch_count before/after the test).  A branch is CREDITED only to a test that
#   * is marked @pytest.mark.oracle (it compares the HIP path with the CPU oracle or a golden
#     fixture -- HIP-vs-HIP self-comparisons are not marked),
#   * consulted a checker while it ran (oracle/consult.py's counter, fixture_io.LOADS): a marked
#     test that consulted neither fails in teardown, so the marker cannot drift from the code, and
#   * passed.
# tests/test_gpu_zz_launch_branches.py then checks that credited tests reached every branch.
BRANCH_HITS = {}          # branch name -> [credited (oracle, passed) test node ids]
BRANCH_OTHER = {}         # branch name -> [other test node ids that reached it]
COLLECTED_FILES = set()   # basenames of the test files this session collected


def pytest_collection_modifyitems(session, config, items):
    for it in items:
        COLLECTED_FILES.add(os.path.basename(str(it.fspath)))


@pytest.hookimpl(hookwrapper=True)
def pytest_runtest_makereport(item, call):
    outcome = yield
    rep = outcome.get_result()
    if rep.when == "call":
        item._flame_call_passed = rep.passed


def _checker_consultations():
    n = 0
    try:
        from oracle import consult
        n += consult.count
    except ImportError:
        pass
    import fixture_io
    return n + fixture_io.LOADS


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
    consulted_before = _checker_consultations()
    yield
    after = _native.launch_branch_counts()
    consulted = _checker_consultations() > consulted_before
    marked = request.node.get_closest_marker("oracle") is not None
    passed = getattr(request.node, "_flame_call_passed", False)
    credit = marked and consulted and passed
    for name, n in after.items():
        BRANCH_HITS.setdefault(name, [])
        BRANCH_OTHER.setdefault(name, [])
        if n > before.get(name, 0):
            (BRANCH_HITS if credit else BRANCH_OTHER)[name].append(request.node.nodeid)
    if marked and passed and not consulted:
        pytest.fail(f"{request.node.nodeid} is marked oracle but consulted neither the CPU oracle nor a "
                    "golden fixture", pytrace=False)
