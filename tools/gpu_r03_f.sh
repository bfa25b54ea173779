#!/bin/bash
# Round 3, step F: full-size parity on EVERY element (C3, C4 x 3, C5) against the C oracle.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03f; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -s --durations=6 --timeout 600 --timeout-method thread -k "full_size" > $OUT/pytest_full.log 2>&1 || { tail -40 $OUT/pytest_full.log; exit 1; }
grep -E "PASS|FAIL|c4/|passed|failed|s call" $OUT/pytest_full.log | tail -20
