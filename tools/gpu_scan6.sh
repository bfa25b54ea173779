#!/bin/bash
# Deferred (batched per workgroup) write-through stores vs per-chunk write-through stores.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1
run() {
  local nm=$1; shift
  timeout -k 10 500 python tools/kernel_sweep.py --rounds 3 --reps 3 --out $OUT/scan6_$nm.json "$@" > $OUT/scan6_$nm.log 2>&1
  local rc=$?; echo "== $nm rc=$rc"; grep -E "median|differs" $OUT/scan6_$nm.log
  return $rc
}
V=stplain:tiled,base:tiled,wgc2d:tiled,wgc4d:tiled,wgc8d:tiled,nostore:tiled
run bf16_64x125M --dtype bf16 --clients 64 --params 125000000 --variants $V &&
run c3 --dtype f32 --clients 1024 --params 25000000 --variants $V
