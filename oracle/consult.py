"""Consultation counter for the CPU checkers (TEST INFRASTRUCTURE ONLY).

Every checker entry point under ``oracle/`` -- the C restatement behind ``oracle.lib()``, the
torch op sequence of ``OracleFedOPT._adapt_torch`` and ``torch_cpu``'s reference loops -- calls
``note()``.  ``tests/conftest.py`` reads ``count`` before and after each GPU test: a test marked
``@pytest.mark.oracle`` must have consulted a checker (or loaded a golden fixture), and only such
tests credit the launch branches they reached (tests/test_gpu_zz_launch_branches.py).
"""

count = 0


def note() -> None:
    global count
    count += 1
