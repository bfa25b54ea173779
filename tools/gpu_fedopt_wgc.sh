#!/bin/bash
# FedOPT with 8 chunks per workgroup (outputs held in LDS, one store burst): GPU FedOPT tests,
# C4 bench for the three variants, kernel trace + PMC passes for FedAdam.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/opt; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
fatal() { rc=$1; [ "$rc" -ge 124 ] || [ "$rc" -gt 128 ]; }
step() {
  local tag=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc"; tail -${TAIL:-1} $OUT/$tag.log | cut -c1-300
  if fatal $rc || [ $rc -ne 0 ]; then exit $rc; fi
  return 0
}
TAIL=3 step pytest_fedopt 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -k "fedopt or fedadam or fedyogi or fedadagrad or c4 or eager or subset"
for w in fedadam fedyogi fedadagrad; do
  step bench_$w 400 python bench.py --workload $w --steps 10 --warmup 3
done
step prof_fedadam 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_fedadam -o run -- \
    python bench.py --workload fedadam --steps 10 --warmup 2 --cpu-clients 0
rm -f $OUT/prof_fedadam/run_kernel_trace.csv
for C in FETCH_SIZE WRITE_SIZE; do
  step pmcopt_$C 300 timeout -s KILL 280 rocprofv3 --pmc $C --kernel-include-regex fedopt --output-format csv \
      -d $OUT/pmcopt_$C -o run -- python bench.py --workload fedadam --steps 3 --warmup 1 --cpu-clients 0
done
cp profiles/traffic.json $OUT/traffic.json
python tools/pmc_traffic.py --fetch $OUT/pmcopt_FETCH_SIZE --write $OUT/pmcopt_WRITE_SIZE --kernel fedopt \
    --name flame_fedopt_reduce_adapt --clients 1024 --params 25000000 --itemsize 4 --extra-arrays 8 --layout slab \
    --out $OUT/traffic.json > $OUT/pmc_traffic.log 2>&1; tail -2 $OUT/pmc_traffic.log | cut -c1-400
exit 0
