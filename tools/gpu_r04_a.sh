#!/bin/bash
# Round 4, first box run on the stripped kernel source: GPU suite (new launch-branch tests
# + guard), smoke, default bench, FedBuff top bench (now low-residency through the
# kernel-argument launch).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04a; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
step() {
  local tag=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc"; tail -${TAIL:-1} $OUT/$tag.log | cut -c1-600
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi   # 1 = test failures: keep going
  return 0
}
TAIL=12 step pytest_gpu 1000 python -u -m pytest tests -m gpu -q -rf --durations=8 --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench_default 600 python bench.py
step bench_fedbuff 300 python bench.py --workload fedbuff --steps 10 --warmup 3
exit 0
