#!/bin/bash
# Round 4: the hierarchy kernel with the next middle's first batch in flight across the epilogue
# (FLAME_HNX, sweep source) A/B against the shipped configuration, bitwise-checked, + its
# attribution; then the full GPU suite (launch-branch guard).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04c; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
step() {
  local tag=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc"; tail -${TAIL:-1} $OUT/$tag.log | cut -c1-300
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
TAIL=6 step hier_hnx_ab 400 python -u tools/hier_sweep.py --mid-layout tiled --rounds 5 \
    --variants build/diag/lib_base.so,build/diag/lib_hnx.so,rprobe
TAIL=30 step hier_attrib_hnx 300 python -u tools/hier_attrib.py --variant hnx --reps 5 --out $OUT/hier_attrib_hnx.json
TAIL=8 step pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf --durations=5 --timeout 300 --timeout-method thread
exit 0
