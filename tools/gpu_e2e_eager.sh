#!/bin/bash
# End-to-end eager top aggregator (per-arrival do() through DeviceUpdateCache) vs the copy pipeline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for cfg in "eager slab" "eager hbm" "copy slab"; do set -- $cfg
  timeout -k 10 300 python bench.py --cpu-clients 0 --e2e --e2e-mode $1 --e2e-placement $2 --steps 3 --warmup 1 \
      > gpurun_out/e2e_$1_$2.log 2>&1 || exit 1
  echo "$cfg $(tail -1 gpurun_out/e2e_$1_$2.log | grep -o '"ms_per_step": [0-9.]*\|"host_read_GBps": [0-9.]*' | tr '\n' ' ')"
done
