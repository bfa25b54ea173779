#!/bin/bash
# PMC pair (FETCH_SIZE, WRITE_SIZE; one counter per run, no trace domains) for the eager FedOPT
# chain kernel -> a traffic.json entry (64 arrivals + base/cur/m/v read + base/m/v/cur written).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04chp; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp FLAME_BENCH_SETTLE=0
cp profiles/traffic.json $OUT/traffic.json
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex fedopt_chain --output-format csv -d $OUT/pmc_$C -o run -- \
      python bench.py --workload fedadam_eager --steps 3 --warmup 1 > $OUT/pmc_$C.log 2>&1
  rc=$?; echo "pmc $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python tools/pmc_traffic.py --fetch $OUT/pmc_FETCH_SIZE --write $OUT/pmc_WRITE_SIZE --kernel fedopt_chain \
    --name flame_fedopt_chain --clients 64 --params 25000000 --itemsize 4 --extra-arrays 8 --layout slab \
    --workload fedadam_eager_chain --out $OUT/traffic.json | cut -c1-400
