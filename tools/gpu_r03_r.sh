#!/bin/bash
# FedOPT split launch (FedAvg reduce, then a no-client adaptive step) vs the fused launch: bitwise
# test, then config 4 A/B/A/B in one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03r; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
step() {
  local tag=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc"; tail -${TAIL:-1} $OUT/$tag.log | cut -c1-600
  if [ $rc -ne 0 ]; then exit $rc; fi
  return 0
}
TAIL=3 step pytest_split 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k split_launch --timeout 200 --timeout-method thread
for i in 1 2; do
  for sp in 0 1; do
    step fedadam_split${sp}_$i 300 env FLAME_AMD_FEDOPT_SPLIT=$sp python bench.py --workload fedadam --steps 10 --warmup 3 --cpu-clients 0
  done
done
step fedyogi_split1 300 env FLAME_AMD_FEDOPT_SPLIT=1 python bench.py --workload fedyogi --steps 10 --warmup 3 --cpu-clients 0
step fedyogi_split0 300 env FLAME_AMD_FEDOPT_SPLIT=0 python bench.py --workload fedyogi --steps 10 --warmup 3 --cpu-clients 0
exit 0
