#!/bin/bash
# Output-store experiments: nt stores / no store (diagnostic) vs base, N=64 bf16 and the C3 headline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1
run() {
  local nm=$1; shift
  timeout -k 10 400 python tools/kernel_sweep.py --rounds 3 --reps 5 --out $OUT/scan2_$nm.json "$@" > $OUT/scan2_$nm.log 2>&1
  local rc=$?; echo "== $nm rc=$rc"; grep -E "median" $OUT/scan2_$nm.log
  return $rc
}
run bf16_64x15M  --dtype bf16 --clients 64 --params 15625000 --variants base,stnt,nostore,base:tiled,stnt:tiled,nostore:tiled,probe &&
run bf16_64x125M --dtype bf16 --clients 64 --params 125000000 --variants base:tiled,stnt:tiled,nostore:tiled,probe &&
run f32_1024x25M --dtype f32 --clients 1024 --params 25000000 --variants base:tiled,stnt:tiled,probe
