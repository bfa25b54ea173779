#!/bin/bash
# Round 3, step I: egress + config 1 after the decoder changes (fresh payloads).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03i; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_egress.py tests/test_gpu_slab_write.py tests/test_gpu_parity.py tests/test_gpu_shm.py -m gpu -q --timeout 200 --timeout-method thread -k "egress or slab or decode or payload or shm or wire" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -u tools/decode_bench.py > $OUT/decode_bench.log 2>&1 || { tail -20 $OUT/decode_bench.log; exit 1; }
cat $OUT/decode_bench.log
timeout -k 10 300 python -u tools/egress_bench.py > $OUT/egress_bench.log 2>&1 || { tail -20 $OUT/egress_bench.log; exit 1; }
cat $OUT/egress_bench.log
timeout -k 10 300 python -u tools/c1_latency.py --profile > $OUT/c1_latency.log 2>&1 || { tail -20 $OUT/c1_latency.log; exit 1; }
head -50 $OUT/c1_latency.log
