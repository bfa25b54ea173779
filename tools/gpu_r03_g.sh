#!/bin/bash
# Round 3, step G: sub-row region probe (hierarchy kernel question) + bench.py N>1 rehearsal
# (2 gloo ranks sharing the GPU) after the round's changes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03g; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 300 python -u tools/subrow_probe.py > $OUT/subrow_probe.log 2>&1 || { tail -20 $OUT/subrow_probe.log; exit 1; }
cat $OUT/subrow_probe.log
timeout -k 10 900 bash tools/gpu_multirank.sh > $OUT/multirank.log 2>&1 || { tail -30 $OUT/multirank.log; exit 1; }
cat $OUT/multirank.log | cut -c1-300
