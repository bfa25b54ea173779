#!/bin/bash
# Sharded product paths on a 1-GPU box: GPU parity tests (two gloo ranks share cuda:0), the
# RCCL code path as a world-1 group (bench --force-shard), a gloo 2-rank rehearsal of the
# N>1 bench, and a kernel trace of one --force-shard FedAvg run.
# Stops at the first fault / abort / timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1
fatal() { rc=$1; [ "$rc" -ge 124 ] || [ "$rc" -gt 128 ]; }
step() {  # step <tag> <timeout> <cmd...>
  local tag=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc"; tail -${TAIL:-2} $OUT/$tag.log
  if fatal $rc; then exit $rc; fi
  return 0
}

TAIL=6 step shard_tests 400 python -u -m pytest tests/test_gpu_shard.py -x -v --timeout 200 --timeout-method thread
[ -n "${FULL:-}" ] && TAIL=4 step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread

export MASTER_ADDR=127.0.0.1
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541"
step force_shard_fedavg 400 $TR bench.py --force-shard --steps 10 --warmup 3
step force_shard_fedadam 400 $TR bench.py --force-shard --workload fedadam --steps 5 --warmup 2
step force_shard_hier 600 $TR bench.py --force-shard --workload hier_fedbuff --steps 5 --warmup 2
step force_shard_hier_sync 600 $TR bench.py --force-shard --workload hier_fedbuff --hier-mode sync --steps 5 --warmup 2

export FLAME_BENCH_BACKEND=gloo
G2="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29543"
step gloo2_fedavg 300 $G2 bench.py --gpus 2 --clients 64 --params 2000000 --steps 3 --warmup 1
step gloo2_fedadam 300 $G2 bench.py --gpus 2 --clients 64 --params 2000000 --steps 3 --warmup 1 --workload fedadam
step gloo2_hier 300 $G2 bench.py --gpus 2 --clients 256 --params 1000000 --steps 3 --warmup 1 --workload hier_fedbuff
unset FLAME_BENCH_BACKEND

if [ -n "${PROF:-}" ]; then
  cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
  RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_PORT=29545 step prof_force_shard 400 \
      rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_shard -o run -- \
      python bench.py --force-shard --steps 10 --warmup 2
  rm -f $OUT/prof_shard/run_kernel_trace.csv
fi
exit 0
