#!/bin/bash
# Process-to-process variance on one box: config 4 (FedAdam) and config 3, 4 processes each, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03v; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
for i in 1 2 3 4; do
  for w in fedadam fedavg; do
    timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 3 --cpu-clients 0 > $OUT/${w}_$i.log 2>&1 || { echo "$w $i failed"; tail -5 $OUT/${w}_$i.log; exit 1; }
    python - "$OUT/${w}_$i.log" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l); r = d["roofline"]
print(sys.argv[1].split("/")[-1], round(d["ms_per_step"], 3), round(r["kernel_ms"], 3), round(r["frac"], 4),
      round(r.get("measured_read_ceiling_GBps") or 0, 1))
PY
  done
done
