#!/bin/bash
# Quick GPU check: the named pytest selection (-k), logs under gpurun_out/quick.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/quick; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -k "${1:-golden}" > $OUT/pytest.log 2>&1
rc=$?; tail -5 $OUT/pytest.log; exit $rc
