#!/bin/bash
# Size / client-count scan of flame_agg_reduce against the streaming-read probe at equal bytes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1
run() {  # name, args...
  local nm=$1; shift
  timeout -k 10 300 python tools/kernel_sweep.py --rounds 3 --reps 5 --out $OUT/scan_$nm.json "$@" > $OUT/scan_$nm.log 2>&1
  local rc=$?; echo "== $nm rc=$rc"; grep -E "median" $OUT/scan_$nm.log
  return $rc
}
run bf16_64x15M   --dtype bf16 --clients 64   --params 15625000  --variants base,c16_2,b128,b512,probe &&
run bf16_64x250M  --dtype bf16 --clients 64   --params 250000000 --variants base,c16_2,probe &&
run bf16_1024x1M  --dtype bf16 --clients 1024 --params 1000000   --variants base,c16_2,probe &&
run f32_1024x1M   --dtype f32  --clients 1024 --params 1000000   --variants base,b128,probe &&
run f32_64x8M     --dtype f32  --clients 64   --params 7812500   --variants base,b128,b512,probe
