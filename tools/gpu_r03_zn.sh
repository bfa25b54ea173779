#!/bin/bash
# Round 3: FedDyn's round kernel and 64-client reductions at lower residency.  Needs build/variants.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03zn; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
step() {
  local tag=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc"; tail -${TAIL:-1} $OUT/$tag.log | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
  return 0
}
TAIL=8 step feddyn_occ 600 python -u tools/feddyn_sweep.py --variants base,dynocc2,dynocc2cu2,dynocc2cu3,dynocc3cu2,dynocc4cu2 --params 6000000 --rounds 4
TAIL=3 step c64_lomin 400 python -u tools/kernel_sweep.py --clients 64 --params 100000000 --rounds 3 --reps 3 \
  --out $OUT/c64.json --variants base:tiled,lomin32:tiled,rprobe
TAIL=3 step b64_lomin 400 python -u tools/kernel_sweep.py --dtype bf16 --clients 64 --params 200000000 --rounds 3 --reps 3 \
  --out $OUT/b64.json --variants base:tiled,lomin32:tiled,rprobe
exit 0
