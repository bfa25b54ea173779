#!/bin/bash
# FedDyn one-pass round and the synchronous hierarchy: rocprofv3 kernel-trace summaries,
# then PMC traffic passes (FETCH_SIZE / WRITE_SIZE in separate runs, no trace domains).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_feddyn -o run -- \
    python bench.py --workload feddyn --steps 10 --warmup 2 > $OUT/prof_feddyn.log 2>&1 \
    || { echo "trace rc=$?"; tail -5 $OUT/prof_feddyn.log; exit 1; }
tail -1 $OUT/prof_feddyn.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_hsync -o run -- \
    python bench.py --workload hier_fedbuff --hier-mode sync --steps 10 --warmup 2 --cpu-clients 0 > $OUT/prof_hsync.log 2>&1 \
    || { echo "trace rc=$?"; tail -5 $OUT/prof_hsync.log; exit 1; }
tail -1 $OUT/prof_hsync.log | cut -c1-400
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex feddyn_kernel --output-format csv \
      -d $OUT/pmcdyn_$C -o run -- python bench.py --workload feddyn --steps 3 --warmup 1 > $OUT/pmcdyn_$C.log 2>&1 \
      || { echo "pmc $C rc=$?"; tail -5 $OUT/pmcdyn_$C.log; exit 1; }
done
cp profiles/traffic.json $OUT/traffic.json
# algorithmic bytes (3N + 3) P s: N = 512 update reads, 512 history reads, 512 history writes, base / avg / cld
python tools/pmc_traffic.py --fetch $OUT/pmcdyn_FETCH_SIZE --write $OUT/pmcdyn_WRITE_SIZE --kernel feddyn_kernel \
    --name flame_feddyn_round --clients 512 --params 25000000 --itemsize 4 --extra-arrays 1027 --layout slab \
    --out $OUT/traffic.json
rm -f $OUT/prof_feddyn/run_kernel_trace.csv $OUT/prof_hsync/run_kernel_trace.csv
