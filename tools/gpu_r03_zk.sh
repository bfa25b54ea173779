#!/bin/bash
# Round 3: cheaper bf16 arithmetic (FLAME_BF16_HI / FLAME_BF16_PK) in the hierarchy kernel and the
# bf16 reduction, bitwise-checked against the base build in each sweep.  Needs build/variants, hvariants.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03zk; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
step() {
  local tag=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc"; tail -${TAIL:-1} $OUT/$tag.log | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
  return 0
}
TAIL=8 step hier_bf16_sweep 500 python -u tools/hier_sweep.py --rounds 3 --reps 3 --mid-layout tiled \
  --variants base,bhi,bpk,bpkcu4,bpkcu5,bpkcu8,rprobe
TAIL=5 step c3_bf16_sweep 500 python -u tools/kernel_sweep.py --dtype bf16 --rounds 3 --reps 3 --out $OUT/c3_bf16.json \
  --variants base:tiled,bpk:tiled,bpklo3:tiled,rprobe
exit 0
