#!/bin/bash
# Round 3: fewer loads in flight per CU.  C3 reduction at 2-4 workgroups per CU and the hierarchy
# kernel with software-pipelined client batches, interleaved against their region probes (2 per CU,
# 6 loads per lane).  Needs build/variants and build/hvariants (drop them from .gpurunignore first).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03zd; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
step() {
  local tag=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc"; tail -${TAIL:-1} $OUT/$tag.log | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
  return 0
}
TAIL=14 step c3_occ_sweep 500 python -u tools/kernel_sweep.py --rounds 3 --reps 3 --out $OUT/c3_occ_sweep.json \
  --variants base:tiled,occ2cu6:tiled,occ2cu8:tiled,occ2cu4:tiled,occ2cu12:tiled,occ3cu4:tiled,occ3cu6:tiled,occ4cu4:tiled,occ2pipe3:tiled,occ2pipe4:tiled,rprobe
TAIL=8 step hier_pipe_sweep 500 python -u tools/hier_sweep.py --rounds 3 --reps 3 --mid-layout tiled \
  --variants base,pipe3,pipe4,pipe6,pipe2,rprobe
exit 0
