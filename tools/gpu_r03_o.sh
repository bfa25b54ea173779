#!/bin/bash
# C pickle VM on the box: ingest-side GPU tests, config-1 round latency (fresh payloads, with
# the Python loop for comparison), the wire end-to-end mode (100 MB payloads decoded per insert).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03o; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
step() {
  local tag=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc"; tail -${TAIL:-1} $OUT/$tag.log | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
  return 0
}
TAIL=3 step pytest_ingest 600 python -u -m pytest tests/test_gpu_shm.py tests/test_gpu_slab_write.py tests/test_gpu_egress.py \
    tests/test_pickle_vm.py tests/test_ingest.py -q --timeout 300 --timeout-method thread
TAIL=8 step c1_c 300 python -u tools/c1_latency.py --profile
TAIL=6 step c1_py 300 env FLAME_AMD_PICKLE_VM=py python -u tools/c1_latency.py
TAIL=6 step c1_c_2 300 python -u tools/c1_latency.py
TAIL=2 step decode_bench 300 python -u tools/decode_bench.py
TAIL=2 step e2e_wire 400 python bench.py --e2e --e2e-mode wire --steps 5 --warmup 2 --cpu-clients 0
exit 0
