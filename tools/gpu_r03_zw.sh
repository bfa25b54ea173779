#!/bin/bash
# After the single-middle low-residency hierarchy launch: GPU suite, smoke, the async FedBuff bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03zw; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -q -x --timeout 600 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -10 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python bench.py --workload fedbuff --steps 10 --warmup 3 --cpu-clients 0 > $OUT/bench_fedbuff.log 2>&1 || { tail -10 $OUT/bench_fedbuff.log; exit 1; }
tail -1 $OUT/bench_fedbuff.log | cut -c1-600
