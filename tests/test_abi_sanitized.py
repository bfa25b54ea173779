"""The product library's host side under ASan + UBSan (SURVEY.md §5 "race detection /
sanitizers"): tests/abi_asan builds libflame_amd.so with its HOST code instrumented
(-Xarch_host -fsanitize=address,undefined; device code untouched) and drives every
C-ABI entry point's argument validation -- NULL tables, bad counts, unknown flags,
metadata blocks and table offsets out of range, 20,000 randomized invalid argmeta
calls -- which must be refused with an error code and message, sanitizer-clean.
Runs on the CPU (nothing reaches HIP)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc") or shutil.which("make") is None,
                    reason="hipcc / make not available")
def test_abi_validation_under_asan_ubsan(tmp_path):
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "abi_asan"), f"OUT={tmp_path}"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "abi asan OK" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr
