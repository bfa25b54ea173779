#!/bin/bash
# Round 3: the hierarchy kernel with one double-buffered arrival stream across middles (FLAME_HXP),
# bitwise-checked against the base build; own middles (tiled) and fetched.  Needs build/hvariants.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03zs; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 500 python -u tools/hier_sweep.py --rounds 3 --reps 3 --mid-layout tiled \
  --variants base,hxp2,hxp4,hxp8,hxp16,rprobe > $OUT/hier_hxp_sweep.log 2>&1 || { tail -20 $OUT/hier_hxp_sweep.log; exit 1; }
tail -7 $OUT/hier_hxp_sweep.log
