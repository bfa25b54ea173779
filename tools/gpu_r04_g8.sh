#!/bin/bash
# The N = 8 bench path rehearsed on the final tree: 8 gloo ranks sharing cuda:0 (the driver's
# 8-GPU run uses RCCL, one GPU per rank), self-check + settle included.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04g8; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp MASTER_ADDR=127.0.0.1 FLAME_BENCH_BACKEND=gloo
G8="python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29561"
timeout -k 10 600 $G8 bench.py --gpus 8 --clients 64 --params 2000000 --steps 3 --warmup 1 > $OUT/gloo8_fedavg.log 2>&1
rc=$?; echo "gloo8_fedavg rc=$rc"; grep '^{' $OUT/gloo8_fedavg.log | cut -c1-250; exit $rc
