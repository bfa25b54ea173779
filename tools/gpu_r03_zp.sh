#!/bin/bash
# The N>1 code paths with the low-residency kernels at sizes that take them (>= 64 clients, >= 4,096
# chunks per wave): bench --force-shard (world-1 RCCL group, 3 waves, in-place gathers) for FedAvg and
# FedAdam at config 3 size, and 2 gloo ranks sharing the GPU (bench's N=2 command line, 128 clients x
# 25M per rank).  Logs under gpurun_out/r03zp.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03zp; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
step() {
  local tag=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc"; tail -${TAIL:-1} $OUT/$tag.log | cut -c1-330
  if [ $rc -ne 0 ]; then tail -20 $OUT/$tag.log; exit $rc; fi
  return 0
}
step force_shard_fedavg 400 python bench.py --force-shard --steps 10 --warmup 3 --cpu-clients 0
step force_shard_fedadam 400 python bench.py --force-shard --workload fedadam --steps 10 --warmup 3 --cpu-clients 0
export FLAME_BENCH_BACKEND=gloo
step gloo2_fedavg 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29537 bench.py --gpus 2 --clients 128 --params 25000000 --steps 3 --warmup 1
step gloo2_fedadam 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29538 bench.py --gpus 2 --workload fedadam --clients 128 --params 25000000 --steps 3 --warmup 1
exit 0
