#!/bin/bash
# Round-2 closing session: the whole GPU suite, smoke(), the default bench (config 3, the
# driver's command) with its kernel trace, config 4 / 5 benches.  Logs under gpurun_out/final.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/final; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
fatal() { rc=$1; [ "$rc" -ge 124 ] || [ "$rc" -gt 128 ]; }
step() {
  local tag=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc"; tail -${TAIL:-1} $OUT/$tag.log | cut -c1-300
  if fatal $rc || [ $rc -ne 0 ]; then exit $rc; fi
  return 0
}
TAIL=3 step pytest_gpu 900 python -u -m pytest tests -m gpu -q --durations=5 --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench_default 600 python bench.py
step prof_default 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_default -o run -- \
    python bench.py --cpu-clients 0
rm -f $OUT/prof_default/run_kernel_trace.csv
step bench_fedadam 400 python bench.py --workload fedadam --steps 10 --warmup 3 --cpu-clients 0
step bench_hier 400 python bench.py --workload hier_fedbuff --steps 20 --warmup 5 --cpu-clients 0
exit 0
