#!/bin/bash
# Round 3: FedOPT residency / unroll variants, 16-bit unroll of the low-occupancy reduction, the
# row layout with and without it.  Needs build/variants.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03zg; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
step() {
  local tag=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc"; tail -${TAIL:-1} $OUT/$tag.log | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
  return 0
}
TAIL=10 step c4_sweep 500 python -u tools/kernel_sweep.py --kernel fedadam --rounds 3 --reps 3 --out $OUT/c4_sweep.json \
  --variants base:tiled,optwgc4cu3:tiled,optwgc4cu2:tiled,optwgc8cu3:tiled,optwgc8cu4:tiled,optwgc6cu3:tiled,optwgc3cu3:tiled,optwgc2cu3:tiled,rprobe
TAIL=5 step c3_bf16_sweep 500 python -u tools/kernel_sweep.py --dtype bf16 --rounds 3 --reps 3 --out $OUT/c3_bf16_sweep.json \
  --variants base:tiled,lo16_3:tiled,lo16_6:tiled,lo0:tiled
TAIL=4 step c3_rows_sweep 500 python -u tools/kernel_sweep.py --rounds 3 --reps 3 --out $OUT/c3_rows_sweep.json \
  --variants base,lo0,probe
exit 0
