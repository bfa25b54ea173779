#!/bin/bash
# Round 3, step J: full GPU suite after the cache / slab-view trims, config 1 latency.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03j; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --durations=5 --timeout 600 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python -u tools/c1_latency.py --profile > $OUT/c1_latency.log 2>&1 || { tail -20 $OUT/c1_latency.log; exit 1; }
head -45 $OUT/c1_latency.log
