#!/bin/bash
# Round 4: the N>1 bench self-check rehearsed (RCCL world-1 --force-shard at full size, gloo
# 2 and 8 ranks sharing cuda:0), C4's variant spread in one process, C5 kernel attribution.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04b; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp MASTER_ADDR=127.0.0.1
step() {
  local tag=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc"; grep '^{' $OUT/$tag.log | cut -c1-300; tail -${TAIL:-1} $OUT/$tag.log | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
  return 0
}
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541"
step rccl1_fedavg 400 $TR bench.py --force-shard --steps 10 --warmup 3
step rccl1_fedadam 400 $TR bench.py --force-shard --workload fedadam --steps 5 --warmup 2
step rccl1_hier 600 $TR bench.py --force-shard --workload hier_fedbuff --steps 5 --warmup 2
step rccl1_hier_sync 600 $TR bench.py --force-shard --workload hier_fedbuff --hier-mode sync --steps 5 --warmup 2
export FLAME_BENCH_BACKEND=gloo
G2="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29543"
step gloo2_fedavg 300 $G2 bench.py --gpus 2 --clients 64 --params 2000000 --steps 3 --warmup 1
step gloo2_fedyogi 300 $G2 bench.py --gpus 2 --clients 64 --params 2000000 --steps 3 --warmup 1 --workload fedyogi
step gloo2_hier 300 $G2 bench.py --gpus 2 --clients 256 --params 1000000 --steps 3 --warmup 1 --workload hier_fedbuff
step gloo2_hier_sync_fetched 300 $G2 bench.py --gpus 2 --clients 256 --params 1000000 --steps 3 --warmup 1 --workload hier_fedbuff --hier-mode sync --hier-middles fetched
G8="python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29547"
step gloo8_fedavg 400 $G8 bench.py --gpus 8 --clients 64 --params 1000000 --steps 3 --warmup 1
step gloo8_hier 400 $G8 bench.py --gpus 8 --clients 256 --params 1000000 --steps 3 --warmup 1 --workload hier_fedbuff
unset FLAME_BENCH_BACKEND
step fedadam_eager 300 python bench.py --workload fedadam_eager --steps 5 --warmup 2
TAIL=3 step fedbuff_ab_f32 300 python -u tools/fedbuff_sweep.py --variants build/diag/lib_base.so,flame_amd/libflame_amd.so --rounds 6
TAIL=3 step fedbuff_ab_bf16 300 python -u tools/fedbuff_sweep.py --dtype bf16 --variants build/diag/lib_base.so,flame_amd/libflame_amd.so --rounds 6
TAIL=2 step fedopt_spread 500 python -u tools/fedopt_spread.py --rounds 9
TAIL=40 step hier_attrib 400 python -u tools/hier_attrib.py --reps 5 --out $OUT/hier_attrib.json
exit 0
