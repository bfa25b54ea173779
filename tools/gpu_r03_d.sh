#!/bin/bash
# Round 3, step D: payload staging (tests + config 1 latency), config 5 host profile + bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03d; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_slab_write.py tests/test_gpu_parity.py tests/test_gpu_shm.py tests/test_gpu_cache_overflow.py tests/test_gpu_eager_defer.py -m gpu -q --timeout 200 --timeout-method thread -k "slab or decode or ingest or payload or shm or cache or eager or arrivals" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 300 python -u tools/c1_latency.py > $OUT/c1_latency.log 2>&1 || { tail -20 $OUT/c1_latency.log; exit 1; }
cat $OUT/c1_latency.log
for mode in batched per-do; do
  timeout -k 10 300 python -u tools/hier_host_profile.py $mode 40 > $OUT/hier_host_$mode.log 2>&1 || { tail -20 $OUT/hier_host_$mode.log; exit 1; }
  head -30 $OUT/hier_host_$mode.log
done
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --workload hier_fedbuff --steps 20 --warmup 3 --cpu-clients 0 > $OUT/bench_hier_$rep.log 2>&1 || { tail -20 $OUT/bench_hier_$rep.log; exit 1; }
  python - $OUT/bench_hier_$rep.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(d["config"].get("arrivals"), "ms/step %.2f" % d["ms_per_step"], "host_issue %.2f" % d["host_issue_ms_per_step"], "frac %.3f" % d["roofline"]["frac"])
PY
done
