#!/bin/bash
# Is the hierarchy kernel's gap to its probe a 16 MiB-region effect?  The bf16 reduction over 4096
# clients x 6.25M (16 MiB regions, 51 GB) and over 1024 x 25M (4 MiB regions) against the 2-per-CU
# region probe of each.  Needs build/variants (base only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03zl; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 400 python -u tools/kernel_sweep.py --dtype bf16 --clients 4096 --params 6250000 --rounds 3 --reps 3 \
  --out $OUT/r16.json --variants base:tiled,rprobe > $OUT/bf16_4096clients.log 2>&1 || exit $?
tail -2 $OUT/bf16_4096clients.log
timeout -k 10 400 python -u tools/kernel_sweep.py --dtype bf16 --clients 64 --params 400000000 --rounds 3 --reps 3 \
  --out $OUT/r256k.json --variants base:tiled,rprobe > $OUT/bf16_64clients.log 2>&1 || exit $?
tail -2 $OUT/bf16_64clients.log
