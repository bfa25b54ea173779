#!/bin/bash
# Chunks-per-workgroup and deferred-store variants (output-write interleaving experiment).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1
run() {
  local nm=$1; shift
  timeout -k 10 500 python tools/kernel_sweep.py --rounds 3 --reps 3 --out $OUT/scan4_$nm.json "$@" > $OUT/scan4_$nm.log 2>&1
  local rc=$?; echo "== $nm rc=$rc"; grep -E "median|differs" $OUT/scan4_$nm.log
  return $rc
}
V=base:tiled,nostore:tiled,wgc2:tiled,wgc4:tiled,wgc2d:tiled,wgc4d:tiled,wgc8d:tiled
run c3 --dtype f32 --clients 1024 --params 25000000 --variants $V &&
run bf16_64x125M --dtype bf16 --clients 64 --params 125000000 --variants $V &&
run f32_1024x1M_rows --dtype f32 --clients 1024 --params 1000000 --variants base,wgc2,wgc4d
