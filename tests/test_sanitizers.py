"""Host sanitizer run of the C oracle (ASan + UBSan), as SURVEY.md §5 asks of the build."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_oracle_under_asan_ubsan():
    r = subprocess.run(["make", "-s", "-B", "-C", os.path.join(ROOT, "oracle"), "selftest"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "oracle selftest OK" in r.stdout
