#!/bin/bash
# Row-layout FedAvg / FedAdam (clients as separate tensors, what an unmodified role hands
# over): XCD-contiguous chunk map on (default) vs off (FLAME_AMD_XCD_MAP_MIN_CHUNKS huge),
# alternating; the GPU tests that reduce row-layout clients first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/xcd; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread \
    -k "fedavg or reduce or golden or c3 or subset or fedopt or feddyn or scaffold" > $OUT/pytest.log 2>&1 \
    || { tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for i in 1 2 3; do
  for mode in on off; do
    if [ $mode = on ]; then M=4096; else M=1000000000; fi
    for w in fedavg fedadam; do
      FLAME_AMD_XCD_MAP_MIN_CHUNKS=$M timeout -k 10 300 python bench.py --workload $w --layout row --steps 10 --warmup 3 \
          --cpu-clients 0 > $OUT/${w}_${mode}_$i.log 2>&1 || { tail -5 $OUT/${w}_${mode}_$i.log; exit 1; }
      echo "$w $mode $i $(grep -o '"kernel_ms": [0-9.]*' $OUT/${w}_${mode}_$i.log)"
    done
  done
done
exit 0
