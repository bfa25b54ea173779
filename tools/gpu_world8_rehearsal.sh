#!/bin/bash
# The driver's N = 8 bench code path rehearsed on a 1-GPU box: 8 gloo ranks share cuda:0
# (FLAME_BENCH_BACKEND=gloo; the real N = 8 runs use RCCL, one GPU per rank), small sizes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/w8; mkdir -p $OUT
fatal() { rc=$1; [ "$rc" -ge 124 ] || [ "$rc" -gt 128 ]; }
step() {
  local tag=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc"; grep '^{' $OUT/$tag.log | cut -c1-400
  if fatal $rc || [ $rc -ne 0 ]; then tail -5 $OUT/$tag.log; exit $rc; fi
  return 0
}
export FLAME_BENCH_BACKEND=gloo MASTER_ADDR=127.0.0.1
G8="python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29547"
step gloo8_fedavg 400 $G8 bench.py --gpus 8 --clients 64 --params 1000000 --steps 3 --warmup 1
step gloo8_fedadam 400 $G8 bench.py --gpus 8 --clients 64 --params 1000000 --steps 3 --warmup 1 --workload fedadam
step gloo8_hier 400 $G8 bench.py --gpus 8 --clients 256 --params 1000000 --steps 3 --warmup 1 --workload hier_fedbuff
step gloo8_hier_sync 400 $G8 bench.py --gpus 8 --clients 256 --params 1000000 --steps 3 --warmup 1 --workload hier_fedbuff --hier-mode sync
exit 0
