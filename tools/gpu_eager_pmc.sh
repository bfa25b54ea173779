#!/bin/bash
# PMC HBM traffic of the eager FedAvg round (64 x 25M fp32, device-resident): one batched
# launch (--eager-defer on) vs a launch per arrival (off).  FETCH_SIZE / WRITE_SIZE in
# separate passes, kernel trace only.  Logs under gpurun_out/eager_pmc.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/eager_pmc; mkdir -p $OUT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
for D in on off; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex agg_reduce --output-format csv \
        -d $OUT/${D}_$C -o run -- python bench.py --workload fedavg_eager --eager-defer $D --steps 3 --warmup 1 \
        > $OUT/${D}_$C.log 2>&1 || { echo "pmc $D $C rc=$?"; tail -5 $OUT/${D}_$C.log; exit 1; }
  done
done
python tools/eager_pmc_summary.py $OUT > $OUT/summary.txt && cat $OUT/summary.txt
