#!/bin/bash
# Extra bench workloads for DESIGN.md (C4 FedOPT, C5 hierarchical FedBuff shard, end-to-end).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
for W in "--workload fedadam" "--workload fedyogi" "--workload hier_fedbuff --steps 3 --warmup 1" "--e2e --steps 3 --warmup 1"; do
  tag=$(echo $W | tr -d ' -' | cut -c1-30)
  timeout -k 10 600 python bench.py --cpu-clients 0 $W > $OUT/wl_$tag.log 2>&1
  rc=$?; echo "$W rc=$rc"; tail -1 $OUT/wl_$tag.log
  if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then exit $rc; fi
done
