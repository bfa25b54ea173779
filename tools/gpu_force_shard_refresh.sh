#!/bin/bash
# The N>1 product path as a world-1 RCCL group, every sharded workload, current build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/fs; mkdir -p $OUT
export MASTER_ADDR=127.0.0.1
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29549"
for w in "fedavg" "fedadam" "hier_fedbuff" "hier_fedbuff --hier-mode sync"; do
  tag=$(echo $w | tr -d ' -')
  timeout -k 10 400 $TR bench.py --force-shard --workload $w --steps 20 --warmup 5 > $OUT/$tag.log 2>&1 || { tail -5 $OUT/$tag.log; exit 1; }
  echo "$w: $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms": [0-9.]*\|"launches_per_step": [0-9.]*' $OUT/$tag.log | tr '\n' ' ')"
done
exit 0
