#!/bin/bash
# Round 3, step A: slab-insert kernel (tests + timing), slab-fed parity tests, C4 full size x 3 variants.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03a; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_slab_write.py -m gpu -v --timeout 120 --timeout-method thread > $OUT/pytest_slab_write.log 2>&1 || { tail -30 $OUT/pytest_slab_write.log; exit 1; }
tail -3 $OUT/pytest_slab_write.log
timeout -k 10 300 python -u tools/slab_write_bench.py > $OUT/slab_write_bench.log 2>&1 || { tail -30 $OUT/slab_write_bench.log; exit 1; }
cat $OUT/slab_write_bench.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cache_overflow.py tests/test_gpu_shm.py tests/test_gpu_eager_defer.py -m gpu -q --timeout 300 --timeout-method thread -k "slab or cache or shm or eager or ingest or decode" > $OUT/pytest_slabfed.log 2>&1 || { tail -30 $OUT/pytest_slabfed.log; exit 1; }
tail -3 $OUT/pytest_slabfed.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --durations=5 --timeout 400 --timeout-method thread -k "c4_full_size" > $OUT/pytest_c4.log 2>&1 || { tail -30 $OUT/pytest_c4.log; exit 1; }
tail -12 $OUT/pytest_c4.log
