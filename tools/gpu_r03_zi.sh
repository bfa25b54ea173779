#!/bin/bash
# Round 3: client-pointer prefetch (FLAME_SPF) in the reduction core: hierarchy kernel, C3, C4.
# Needs build/variants and build/hvariants.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03zi; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
step() {
  local tag=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc"; tail -${TAIL:-1} $OUT/$tag.log | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
  return 0
}
TAIL=7 step hier_spf_sweep 500 python -u tools/hier_sweep.py --rounds 3 --reps 3 --mid-layout tiled \
  --variants base,spf,spfcu5,spfcu8,spfcu4,rprobe
TAIL=5 step c3_spf_sweep 500 python -u tools/kernel_sweep.py --rounds 3 --reps 3 --out $OUT/c3.json \
  --variants base:tiled,spf:tiled,spflo4:tiled,rprobe
TAIL=4 step c4_spf_sweep 500 python -u tools/kernel_sweep.py --kernel fedadam --rounds 3 --reps 3 --out $OUT/c4.json \
  --variants base:tiled,spf:tiled,rprobe
exit 0
