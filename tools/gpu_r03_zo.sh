#!/bin/bash
# Round 3 final verification with the shipped library: GPU suite, smoke, default bench + kernel trace
# (PART A); C4 x 3, C5, eager (64 arrivals, now on the low-residency path), C2 (PART B).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03zo; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
step() {
  local tag=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc"; tail -${TAIL:-1} $OUT/$tag.log | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
  return 0
}
if [ "${PART:-A}" = A ]; then
TAIL=3 step pytest_gpu 900 python -u -m pytest tests -m gpu -q --durations=5 --timeout 600 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench_default 600 python bench.py
step prof_default 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_default -o run -- \
    python bench.py --cpu-clients 0
rm -f $OUT/prof_default/run_kernel_trace.csv
exit 0
fi
for w in fedadam fedyogi fedadagrad; do
  step bench_$w 400 python bench.py --workload $w --steps 10 --warmup 3 --cpu-clients 0
done
step bench_hier 400 python bench.py --workload hier_fedbuff --steps 20 --warmup 5 --cpu-clients 0
step bench_eager 400 python bench.py --workload fedavg_eager --steps 10 --warmup 3 --cpu-clients 0
step bench_c2 300 python bench.py --clients 256 --params 1000000 --steps 50 --warmup 5 --cpu-clients 0
step bench_scaffold 400 python bench.py --workload scaffold --steps 10 --warmup 3 --cpu-clients 0
exit 0
