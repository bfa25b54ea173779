#!/bin/bash
# Rehearse bench.py's N>1 path on a 1-GPU box: 2 ranks share cuda:0 over gloo (host collectives).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
export FLAME_BENCH_BACKEND=gloo
for W in "--workload fedavg" "--workload fedavg --no-overlap" "--workload fedadam" "--workload hier_fedbuff --clients 256 --params 1000000"; do
  tag=$(echo $W | tr -d ' -')
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29533 bench.py --gpus 2 --clients 64 --params 2000000 --steps 3 --warmup 1 $W > $OUT/mr_$tag.log 2>&1
  rc=$?; echo "$W rc=$rc"; tail -1 $OUT/mr_$tag.log
  if [ $rc -ne 0 ]; then tail -20 $OUT/mr_$tag.log; exit $rc; fi
done
