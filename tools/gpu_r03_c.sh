#!/bin/bash
# Round 3, step C: batched arrivals (tests + config 5 host issue), dtype-default test, shard tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03c; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dtype_matrix.py tests/test_gpu_shard.py tests/test_gpu_slab_write.py tests/test_gpu_shm.py tests/test_gpu_cache_overflow.py -m gpu -q --timeout 200 --timeout-method thread -k "arrivals or float64_default or wave_quantum or shard or slab_write or rccl or feddyn or decode or ingest or payload or shm or cache" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
for mode in batched per-do batched per-do; do
  timeout -k 10 300 python -u bench.py --workload hier_fedbuff --steps 20 --warmup 3 --hier-arrivals $mode --cpu-clients 0 > $OUT/bench_hier_$mode.log 2>&1 || { tail -20 $OUT/bench_hier_$mode.log; exit 1; }
  python - $OUT/bench_hier_$mode.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(d["config"].get("arrivals"), "ms/step %.2f" % d["ms_per_step"], "host_issue %.2f" % d["host_issue_ms_per_step"], "frac %.3f" % d["roofline"]["frac"])
PY
done
timeout -k 10 300 python -u bench.py --workload hier_fedbuff --steps 20 --warmup 3 --force-shard --cpu-clients 0 > $OUT/bench_hier_shard.log 2>&1 || { tail -20 $OUT/bench_hier_shard.log; exit 1; }
tail -1 $OUT/bench_hier_shard.log | cut -c1-400
timeout -k 10 300 python -u tools/c1_latency.py > $OUT/c1_latency.log 2>&1 || { tail -20 $OUT/c1_latency.log; exit 1; }
cat $OUT/c1_latency.log
