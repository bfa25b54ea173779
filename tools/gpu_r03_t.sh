#!/bin/bash
# Config 2 (256 x 1M fp32): bench, and a kernel trace to read the gaps between steps' launches.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03t; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
step() {
  local tag=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc"; tail -${TAIL:-1} $OUT/$tag.log | cut -c1-900
  if [ $rc -ne 0 ]; then exit $rc; fi
  return 0
}
step bench_c2 300 python bench.py --clients 256 --params 1000000 --steps 200 --warmup 20 --cpu-clients 0
step prof_c2 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_c2 -o run -- \
    python bench.py --clients 256 --params 1000000 --steps 200 --warmup 20 --cpu-clients 0
TAIL=30 step gaps 60 python tools/kernel_gaps.py $OUT/prof_c2 agg_reduce
exit 0
