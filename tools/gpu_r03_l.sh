#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03l; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 300 python -u tools/hier_host_profile.py batched 40 --sharded > $OUT/hier_host_sharded.log 2>&1 || { tail -20 $OUT/hier_host_sharded.log; exit 1; }
head -40 $OUT/hier_host_sharded.log
