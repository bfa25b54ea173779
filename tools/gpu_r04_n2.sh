#!/bin/bash
# N>1 paths after the settle step and the chain kernel: RCCL world 1 (force-shard), gloo world 2
# on one GPU (the self-checking sharded lines; FLAME_BENCH_BACKEND=gloo as in gpu_r04_b.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04n2; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp MASTER_ADDR=127.0.0.1
step() { local tag=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $OUT/$tag.log 2>&1; local rc=$?; echo "$tag rc=$rc"; grep '^{' $OUT/$tag.log | cut -c1-200; [ $rc -eq 0 ] || { tail -5 $OUT/$tag.log; exit $rc; }; }
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29551"
step rccl1_fedavg 400 $TR bench.py --force-shard --steps 10 --warmup 3
export FLAME_BENCH_BACKEND=gloo
G2="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29553"
step gloo2_fedavg 300 $G2 bench.py --gpus 2 --clients 64 --params 2000000 --steps 3 --warmup 1
