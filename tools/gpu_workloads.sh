#!/bin/bash
# Extra bench workloads for DESIGN.md (C4 FedOPT, C5 hierarchical FedBuff shard, end-to-end).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
WL=${WORKLOADS:-"fedadam fedyogi hier e2e_zerocopy e2e_copy e2e_pageable e2e_wire e2e_wire_pinned e2e_wire_reference"}
for w in $WL; do
  case $w in
    hier) W="--workload hier_fedbuff --steps 3 --warmup 1";;
    e2e_*) W="--e2e --e2e-mode ${w#e2e_} --steps 3 --warmup 1";;
    *) W="--workload $w";;
  esac
  timeout -k 10 600 python bench.py --cpu-clients 0 $W > $OUT/wl_$w.log 2>&1
  rc=$?; echo "$w rc=$rc"; tail -1 $OUT/wl_$w.log
  if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then exit $rc; fi
done
