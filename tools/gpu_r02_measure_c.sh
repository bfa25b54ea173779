#!/bin/bash
# Round-2 measurement session, part C: config 5 after the LDS-held store groups -- bench,
# kernel trace, PMC traffic passes, the sharded product path (force-shard, world-1 RCCL), the
# middle-layout comparison, then the whole GPU suite.  Logs under gpurun_out/r02c.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r02c; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1
fatal() { rc=$1; [ "$rc" -ge 124 ] || [ "$rc" -gt 128 ]; }
step() {
  local tag=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc"; tail -${TAIL:-1} $OUT/$tag.log | cut -c1-300
  if fatal $rc; then exit $rc; fi
  return 0
}
export TMPDIR=/tmp
step bench_hier 400 python bench.py --workload hier_fedbuff --steps 30 --warmup 5
step bench_hier_sync 400 python bench.py --workload hier_fedbuff --hier-mode sync --steps 30 --warmup 5
step prof_hier 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_hier -o run -- \
    python bench.py --workload hier_fedbuff --steps 10 --warmup 2 --cpu-clients 0
rm -f $OUT/prof_hier/run_kernel_trace.csv
for C in FETCH_SIZE WRITE_SIZE; do
  step pmchier_$C 300 timeout -s KILL 280 rocprofv3 --pmc $C --kernel-include-regex hier_fedbuff --output-format csv \
      -d $OUT/pmchier_$C -o run -- python bench.py --workload hier_fedbuff --steps 3 --warmup 1 --cpu-clients 0
done
cp profiles/traffic.json $OUT/traffic.json
python tools/pmc_traffic.py --fetch $OUT/pmchier_FETCH_SIZE --write $OUT/pmchier_WRITE_SIZE --kernel hier_fedbuff \
    --name flame_hier_fedbuff --clients 4096 --params 15625000 --itemsize 2 --extra-arrays 131 --layout slab \
    --out $OUT/traffic.json > $OUT/pmc_traffic.log 2>&1; tail -2 $OUT/pmc_traffic.log
export MASTER_ADDR=127.0.0.1
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29543"
step shard_hier 500 $TR bench.py --force-shard --workload hier_fedbuff --steps 20 --warmup 5
step shard_hier_sync 500 $TR bench.py --force-shard --workload hier_fedbuff --hier-mode sync --steps 20 --warmup 5
step hier_midlayout 300 python tools/hier_midlayout.py --rounds 6
TAIL=3 step pytest_gpu 900 python -u -m pytest tests -m gpu -q --durations=8 --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
exit 0
