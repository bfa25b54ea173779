#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 500 python tools/kernel_sweep.py --rounds 3 --reps 3 --out $OUT/scan3_c3.json --dtype f32 --clients 1024 \
    --params 25000000 --variants base:tiled,nostore:tiled,probe > $OUT/scan3_c3.log 2>&1
rc=$?; echo "rc=$rc"; grep median $OUT/scan3_c3.log
