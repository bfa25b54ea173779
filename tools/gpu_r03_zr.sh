#!/bin/bash
# The bf16 reduction over 4,096 clients (16 MiB regions) with enough chunks to take the low-residency
# path (12.5M params = 6,104 chunks), against full residency and the 2-per-CU region probe.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03zr; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 500 python -u tools/kernel_sweep.py --dtype bf16 --clients 4096 --params 12500000 --rounds 3 --reps 3 \
  --out $OUT/b4096.json --variants base:tiled,lo0:tiled,rprobe > $OUT/bf16_4096clients_lo.log 2>&1 || exit $?
tail -3 $OUT/bf16_4096clients_lo.log
