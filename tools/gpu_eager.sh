#!/bin/bash
# Eager FedAvg deferral: GPU tests, device-resident eager rounds (defer on/off, A/B/A/B),
# and the end-to-end eager mode (defer on/off).  Logs under gpurun_out/eager.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/eager; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
step() {
  local tag=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc"; tail -${TAIL:-1} $OUT/$tag.log | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
TAIL=3 step pytest 300 python -u -m pytest tests/test_gpu_eager_defer.py tests/test_gpu_parity.py -k "eager or golden_bitwise" -v --timeout 120 --timeout-method thread
for r in 1 2; do
  step dev_on_$r 300 python bench.py --workload fedavg_eager --eager-defer on --steps 10 --warmup 3
  step dev_off_$r 300 python bench.py --workload fedavg_eager --eager-defer off --steps 10 --warmup 3
done
step e2e_on 300 python bench.py --e2e --e2e-mode eager --eager-defer on --steps 5 --warmup 2
step e2e_off 300 python bench.py --e2e --e2e-mode eager --eager-defer off --steps 5 --warmup 2
step prof_on 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_on -o run -- \
    python bench.py --workload fedavg_eager --eager-defer on --steps 10 --warmup 3
rm -f $OUT/prof_on/run_kernel_trace.csv
exit 0
