#!/bin/bash
# HBM ceiling probe + PMC traffic passes (FETCH_SIZE / WRITE_SIZE in separate runs, no trace domains).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python tools/hbm_probe.py > $OUT/probe.log 2>&1 || { echo "probe rc=$?"; exit 1; }
tail -8 $OUT/probe.log
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C --kernel-include-regex agg_reduce --output-format csv \
      -d $OUT/pmc_$C -o run -- python bench.py --steps 3 --warmup 1 --cpu-clients 0 ${BENCH_ARGS:-} > $OUT/pmc_$C.log 2>&1 \
      || { echo "pmc $C rc=$?"; tail -5 $OUT/pmc_$C.log; exit 1; }
done
cp profiles/traffic.json $OUT/traffic.json 2>/dev/null
python tools/pmc_traffic.py --fetch $OUT/pmc_FETCH_SIZE --write $OUT/pmc_WRITE_SIZE --layout slab --out $OUT/traffic.json
# fused FedOPT kernel (C4)
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C --kernel-include-regex fedopt_kernel --output-format csv \
      -d $OUT/pmcopt_$C -o run -- python bench.py --workload fedadam --steps 3 --warmup 1 --cpu-clients 0 > $OUT/pmcopt_$C.log 2>&1 \
      || { echo "pmc opt $C rc=$?"; tail -5 $OUT/pmcopt_$C.log; exit 1; }
done
python tools/pmc_traffic.py --fetch $OUT/pmcopt_FETCH_SIZE --write $OUT/pmcopt_WRITE_SIZE --kernel fedopt_kernel \
    --name flame_fedopt_reduce_adapt --extra-arrays 8 --layout slab --out $OUT/traffic.json
