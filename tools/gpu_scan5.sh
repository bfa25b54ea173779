#!/bin/bash
# Store cache-policy variants and the previous kernel build ("old") vs the current one.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1
run() {
  local nm=$1; shift
  timeout -k 10 500 python tools/kernel_sweep.py --rounds 3 --reps 3 --out $OUT/scan5_$nm.json "$@" > $OUT/scan5_$nm.log 2>&1
  local rc=$?; echo "== $nm rc=$rc"; grep -E "median|differs" $OUT/scan5_$nm.log
  return $rc
}
V=old:tiled,base:tiled,stnt:tiled,stsc1:tiled,stsc01:tiled,stsc01nt:tiled,nostore:tiled,probe
run c3 --dtype f32 --clients 1024 --params 25000000 --variants $V &&
run bf16_64x125M --dtype bf16 --clients 64 --params 125000000 --variants $V
