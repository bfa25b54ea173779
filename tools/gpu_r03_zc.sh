#!/bin/bash
# Tail-effect and occupancy probes (tools/tail_probe.py, tools/occ_probe.py).  Logs under gpurun_out/r03zc.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03zc; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 300 python -u tools/occ_probe.py > $OUT/occ_probe.log 2>&1
rc=$?; cat $OUT/occ_probe.log; exit $rc
