#!/bin/bash
# Config 5 shard (fused hierarchy): rocprofv3 kernel-trace summary, then PMC traffic passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_hier -o run -- \
    python bench.py --workload hier_fedbuff --steps 10 --warmup 2 --cpu-clients 0 > $OUT/prof_hier.log 2>&1 \
    || { echo "trace rc=$?"; tail -5 $OUT/prof_hier.log; exit 1; }
tail -1 $OUT/prof_hier.log
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex hier_fedbuff --output-format csv \
      -d $OUT/pmchier_$C -o run -- python bench.py --workload hier_fedbuff --steps 3 --warmup 1 --cpu-clients 0 > $OUT/pmchier_$C.log 2>&1 \
      || { echo "pmc $C rc=$?"; tail -5 $OUT/pmchier_$C.log; exit 1; }
done
cp profiles/traffic.json $OUT/traffic.json
python tools/pmc_traffic.py --fetch $OUT/pmchier_FETCH_SIZE --write $OUT/pmchier_WRITE_SIZE --kernel hier_fedbuff \
    --name flame_hier_fedbuff --clients 4096 --params 15625000 --itemsize 2 --extra-arrays 131 --layout slab \
    --out $OUT/traffic.json
rm -f $OUT/prof_hier/run_kernel_trace.csv   # 65k slab-fill copies: too big to bring back
