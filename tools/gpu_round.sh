#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel-trace summary.
# Stops at the first fault / abort / timeout (exit >= 124 or signal), continues past plain test failures.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1
fatal() { rc=$1; [ "$rc" -ge 124 ] || [ "$rc" -gt 128 ]; }

python -m flame_amd.build > $OUT/build.log 2>&1 || { echo "build failed"; exit 2; }
make -s -C oracle >> $OUT/build.log 2>&1

timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -m gpu -q -rs ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest_gpu.log
if fatal $rc; then exit $rc; fi

timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $OUT/smoke.log
if fatal $rc; then exit $rc; fi

timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 $OUT/bench.log
if fatal $rc; then exit $rc; fi

if [ -n "${PROF:-}" ]; then
  cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
      python bench.py --cpu-clients 0 --steps 10 --warmup 2 ${BENCH_ARGS:-} > $OUT/prof.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -3 $OUT/prof.log
  rm -f $OUT/prof/run_kernel_trace.csv   # tens of MB; the stats file is what gets committed
fi
exit 0
