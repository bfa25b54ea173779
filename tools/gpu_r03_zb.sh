#!/bin/bash
# Region-size probes for a 1 KiB-tile hierarchy slab (tools/tile_probe.py) and the hierarchy
# bench with its same-process read probes.  Logs under gpurun_out/r03zb.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03zb; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
step() {
  local tag=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc"; tail -${TAIL:-1} $OUT/$tag.log | cut -c1-600
  if [ $rc -ne 0 ]; then exit $rc; fi
  return 0
}
TAIL=12 step tile_probe 300 python -u tools/tile_probe.py
step bench_hier 400 python bench.py --workload hier_fedbuff --steps 20 --warmup 5 --cpu-clients 0
exit 0
