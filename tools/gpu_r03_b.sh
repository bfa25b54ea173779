#!/bin/bash
# Round 3, step B: slab-insert variant sweep (tiles per workgroup x store policy), then C4 full size.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03b; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
for rep in 1 2; do
for v in build/slabvar/lib_t*.so flame_amd/libflame_amd.so; do
  echo "== $v" >> $OUT/slab_sweep.log
  FLAME_AMD_LIB=$PWD/$v timeout -k 10 120 python -u tools/slab_write_bench.py --cases device >> $OUT/slab_sweep.log 2>&1 || { tail -20 $OUT/slab_sweep.log; exit 1; }
done
done
grep -E "==|kernel|torch|2d" $OUT/slab_sweep.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --durations=5 --timeout 400 --timeout-method thread -k "c4_full_size" > $OUT/pytest_c4.log 2>&1 || { tail -30 $OUT/pytest_c4.log; exit 1; }
tail -12 $OUT/pytest_c4.log
