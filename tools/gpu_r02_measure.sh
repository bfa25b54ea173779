#!/bin/bash
# Round-2 measurement session, part A: GPU suite, C3 bench + kernel trace, the N>1 code path
# (world-1 RCCL group) under a kernel trace, gloo two-rank rehearsals.  Logs -> gpurun_out/r02/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r02; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1
fatal() { rc=$1; [ "$rc" -ge 124 ] || [ "$rc" -gt 128 ]; }
step() {  # step <tag> <timeout> <cmd...>
  local tag=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc"; tail -${TAIL:-1} $OUT/$tag.log | cut -c1-300
  if fatal $rc; then exit $rc; fi
  return 0
}
prof() {  # prof <tag> <timeout> <cmd...>: kernel-trace stats of a command
  local tag=$1 lim=$2; shift 2
  (cd /tmp) ; export TMPDIR=/tmp
  step $tag $lim rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$tag -o run -- "$@"
  rm -f $OUT/$tag/run_kernel_trace.csv
}
TAIL=3 step pytest_gpu 900 python -u -m pytest tests -m gpu -v --durations=12 --timeout 300 --timeout-method thread
step bench_c3 400 python bench.py --steps 20 --warmup 5
prof prof_c3 400 python bench.py --cpu-clients 0 --steps 10 --warmup 2
RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29545 \
    prof prof_force_shard_fedavg 400 python bench.py --force-shard --steps 10 --warmup 2
export FLAME_BENCH_BACKEND=gloo
G2="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29543"
step gloo2_fedavg 300 $G2 bench.py --gpus 2 --clients 64 --params 2000000 --steps 3 --warmup 1
step gloo2_fedadam 300 $G2 bench.py --gpus 2 --clients 64 --params 2000000 --steps 3 --warmup 1 --workload fedadam
step gloo2_hier 300 $G2 bench.py --gpus 2 --clients 256 --params 1000000 --steps 3 --warmup 1 --workload hier_fedbuff
step gloo2_hier_sync 300 $G2 bench.py --gpus 2 --clients 256 --params 1000000 --steps 3 --warmup 1 --workload hier_fedbuff --hier-mode sync
unset FLAME_BENCH_BACKEND
exit 0
