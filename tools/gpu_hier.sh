#!/bin/bash
# Hierarchy (config 5 shard): parity tests for flame_hier_fedbuff, then fused vs group bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "hierarchy or middle" --timeout 120 --timeout-method thread > $OUT/pytest_hier.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest_hier.log
[ $rc -eq 0 ] || exit $rc
for mode in ${MODES:-fused group}; do
  timeout -k 10 300 python bench.py --workload hier_fedbuff --hier-mode $mode --cpu-clients 0 ${BENCH_ARGS:-} > $OUT/hier_$mode.log 2>&1
  rc=$?; echo "bench $mode rc=$rc"; tail -1 $OUT/hier_$mode.log
  [ $rc -eq 0 ] || exit $rc
done
