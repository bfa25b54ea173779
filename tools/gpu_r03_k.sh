#!/bin/bash
# Round 3, step K: do_arrivals (defer on/off) tests, sharded config-5 host issue.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03k; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shard.py -m gpu -q --timeout 200 --timeout-method thread -k "arrivals or wave_quantum" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for a in batched per-do; do
timeout -k 10 300 python -u bench.py --workload hier_fedbuff --steps 20 --warmup 3 --force-shard --cpu-clients 0 --hier-arrivals $a > $OUT/bench_hier_shard_$a.log 2>&1 || { tail -20 $OUT/bench_hier_shard_$a.log; exit 1; }
python - $OUT/bench_hier_shard_$a.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(d["config"].get("arrivals"), "ms/step %.2f" % d["ms_per_step"], "host_issue %.2f" % d["host_issue_ms_per_step"], "frac %.3f" % d["roofline"]["frac"])
PY
done
