#!/bin/bash
# Round 3: pointers AND rates prefetched one batch ahead (FLAME_SPF, second version) -- hierarchy,
# the 4096-client bf16 reduction (16 MiB regions), C3 fp32, C4.  Needs build/variants, hvariants.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03zm; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
step() {
  local tag=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc"; tail -${TAIL:-1} $OUT/$tag.log | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
  return 0
}
TAIL=6 step hier_spf2_sweep 500 python -u tools/hier_sweep.py --rounds 3 --reps 3 --mid-layout tiled \
  --variants base,spf2,spf2cu5,spf2cu4,spf2cu8,rprobe
TAIL=3 step bf16_4096_spf2 400 python -u tools/kernel_sweep.py --dtype bf16 --clients 4096 --params 6250000 --rounds 3 --reps 3 \
  --out $OUT/b4096.json --variants base:tiled,spf2:tiled,rprobe
TAIL=3 step c3_spf2 400 python -u tools/kernel_sweep.py --rounds 3 --reps 3 --out $OUT/c3.json --variants base:tiled,spf2:tiled,rprobe
TAIL=3 step c4_spf2 400 python -u tools/kernel_sweep.py --kernel fedadam --rounds 3 --reps 3 --out $OUT/c4.json --variants base:tiled,spf2:tiled,rprobe
exit 0
