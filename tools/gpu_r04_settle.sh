#!/bin/bash
# the next process after a large one: placement or something beside it? (tools/settle_probe.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04se; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-clients 0 > $OUT/bench.log 2>&1 || exit 1
echo bench done
timeout -k 10 300 python -u tools/settle_probe.py --gb 16 --secs 90 --every 3 > $OUT/settle.log 2>&1; rc=$?
grep -v amdgpu.ids $OUT/settle.log | grep -v '^{'
exit $rc
