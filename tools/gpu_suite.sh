#!/bin/bash
# Full GPU suite + the config-5 benches (one-GPU shard and the sharded product path).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1
fatal() { rc=$1; [ "$rc" -ge 124 ] || [ "$rc" -gt 128 ]; }
step() {  # step <tag> <timeout> <cmd...>
  local tag=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc"; tail -${TAIL:-1} $OUT/$tag.log | cut -c1-400
  if fatal $rc; then exit $rc; fi
  return 0
}
TAIL=3 step pytest_gpu 900 python -u -m pytest tests -m gpu -q --durations=8 --timeout 300 --timeout-method thread
step hier_tiled 400 python bench.py --workload hier_fedbuff --steps 10 --warmup 3 --cpu-clients 0
step hier_row 400 python bench.py --workload hier_fedbuff --steps 10 --warmup 3 --cpu-clients 0 --hier-mid-layout row
step feddyn_pp 400 python bench.py --workload feddyn --steps 8 --warmup 2
step feddyn_rows 400 python bench.py --workload feddyn --steps 8 --warmup 2 --feddyn-history rows
step feddyn_pp_shuf 400 python bench.py --workload feddyn --steps 8 --warmup 2 --feddyn-order shuffled
step hier_sync 400 python bench.py --workload hier_fedbuff --hier-mode sync --steps 10 --warmup 3 --cpu-clients 0
export MASTER_ADDR=127.0.0.1
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541"
step shard_hier 500 $TR bench.py --force-shard --workload hier_fedbuff --steps 20 --warmup 5
step shard_hier_sync 500 $TR bench.py --force-shard --workload hier_fedbuff --hier-mode sync --steps 20 --warmup 5
exit 0
