#!/bin/bash
# do_arrivals parity with defer on/off, the sharded hierarchy host profile, and the slab-insert
# kernel's HBM traffic (FETCH_SIZE / WRITE_SIZE in separate passes, no trace domains).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03n; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
step() {
  local tag=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc"; tail -${TAIL:-1} $OUT/$tag.log | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
  return 0
}
TAIL=3 step pytest_arrivals 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k do_arrivals --timeout 120 --timeout-method thread
TAIL=40 step hier_host_sharded 300 python -u tools/hier_host_profile.py batched 40 --sharded
for C in FETCH_SIZE WRITE_SIZE; do
  step pmc_slab_$C 120 rocprofv3 --pmc $C --kernel-include-regex slab_write --output-format csv \
      -d $OUT/pmc_slab_$C -o run -- python tools/slab_write_bench.py --cases device --capacity 16 --reps 8
done
TAIL=20 step traffic_slab 60 python tools/pmc_traffic.py --fetch $OUT/pmc_slab_FETCH_SIZE --write $OUT/pmc_slab_WRITE_SIZE \
    --kernel slab_write --name flame_slab_write --clients 1 --extra-arrays 1 --layout slab_insert --out $OUT/traffic_slab.json
exit 0
