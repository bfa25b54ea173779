#!/bin/bash
# Sharded hierarchy (config 5 shard, world-1 RCCL group): last wave sized to whole rounds of
# resident workgroups (--hier-wave-quantum on) vs the plain 0.9/0.1 split, both modes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/wq; mkdir -p $OUT
fatal() { rc=$1; [ "$rc" -ge 124 ] || [ "$rc" -gt 128 ]; }
step() {
  local tag=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc"; tail -${TAIL:-1} $OUT/$tag.log | cut -c1-200
  if fatal $rc || [ $rc -ne 0 ]; then exit $rc; fi
  return 0
}
TAIL=3 step pytest 300 python -u -m pytest tests/test_gpu_shard.py -q -x --timeout 200 --timeout-method thread
export MASTER_ADDR=127.0.0.1
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29545"
for mode in fused sync; do
  for wq in on off on; do
    step shard_${mode}_$wq 400 $TR bench.py --force-shard --workload hier_fedbuff --hier-mode $mode --hier-wave-quantum $wq --steps 20 --warmup 5
    grep -o '"kernel_ms": [0-9.]*\|"ms_per_step": [0-9.]*\|"wave_elements_per_rank": \[[0-9, ]*\]' $OUT/shard_${mode}_$wq.log | tr '\n' ' '; echo
  done
done
exit 0
