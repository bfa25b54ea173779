#!/bin/bash
# Eager FedOPT rounds: the deferred chain (one flame_fedopt_chain launch per round) vs one fused
# launch per arrival, 64 arrivals x 25M fp32, and the chain under rocprofv3 (kernel trace).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04ch; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
run() { local tag=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $OUT/$tag.log 2>&1; local rc=$?; echo "$tag rc=$rc"; grep '^{' $OUT/$tag.log | cut -c1-260; [ $rc -eq 0 ] || exit $rc; }
for w in fedadam fedyogi fedadagrad; do
  run bench_${w}_eager_chain 300 python bench.py --workload ${w}_eager --steps 10 --warmup 2
done
run bench_fedadam_eager_percall 300 python bench.py --workload fedadam_eager --eager-defer off --steps 5 --warmup 2
run prof_fedadam_eager_chain 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_chain -o run -- \
    python bench.py --workload fedadam_eager --steps 10 --warmup 2
rm -f $OUT/prof_chain/run_kernel_trace.csv
