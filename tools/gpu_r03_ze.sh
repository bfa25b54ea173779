#!/bin/bash
# Round 3: whole client batches (FLAME_TAILB) and fewer loads in flight per CU, for C3 (FedAvg),
# C4 (FedAdam) and the hierarchy kernel, interleaved against their region probes.
# Needs build/variants and build/hvariants (drop them from .gpurunignore first).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03ze; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
step() {
  local tag=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc"; tail -${TAIL:-1} $OUT/$tag.log | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
  return 0
}
TAIL=10 step hier_tailb_sweep 500 python -u tools/hier_sweep.py --rounds 3 --reps 3 --mid-layout tiled \
  --variants base,tailb,tailbpf,tailbcu5,tailbcu7,tailbcu8,tailbcu4,rprobe
TAIL=13 step c3_sweep 500 python -u tools/kernel_sweep.py --rounds 3 --reps 3 --out $OUT/c3_sweep.json \
  --variants base:tiled,tailb:tiled,occ2cu4:tiled,occ2cu4tb:tiled,occ2cu6tb:tiled,occ2cu3:tiled,occ2cu2:tiled,occ2cu5:tiled,occ3cu3:tiled,occ3cu2:tiled,rprobe
TAIL=7 step c4_sweep 500 python -u tools/kernel_sweep.py --kernel fedadam --rounds 3 --reps 3 --out $OUT/c4_sweep.json \
  --variants base:tiled,tailb:tiled,optwgc4:tiled,optwgc4cu6:tiled,optwgc8cu12:tiled,rprobe
exit 0
