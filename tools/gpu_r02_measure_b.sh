#!/bin/bash
# Round-2 measurement session, part B: config 5 (hierarchy) -- bench + kernel trace + PMC
# traffic passes, the in-process variant sweep and middle-layout comparison.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r02; mkdir -p $OUT
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
step bench_hier 400 python bench.py --workload hier_fedbuff --steps 20 --warmup 5
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
step hier_sweep 500 python tools/hier_sweep.py --variants r01,r01:tiled,base,base:tiled,hdiag1,hdiag1:tiled --rounds 4
step hier_midlayout 300 python tools/hier_midlayout.py --rounds 6
exit 0
