#!/bin/bash
# FedAdam bench on one box: product library (8 chunks per workgroup) vs the one-chunk build
# (build/variants/lib_optwgc1.so via FLAME_AMD_LIB), A/B/A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/optab; mkdir -p $OUT
for i in 1 2 3 4 5; do
  for lib in product optwgc1; do
    if [ $lib = product ]; then L=flame_amd/libflame_amd.so; else L=build/variants/lib_$lib.so; fi
    FLAME_AMD_LIB=$L timeout -k 10 300 python bench.py --workload fedadam --steps 10 --warmup 3 --cpu-clients 0 \
        > $OUT/${lib}_$i.log 2>&1 || exit $?
    echo "$lib $i $(grep -o '"kernel_ms": [0-9.]*' $OUT/${lib}_$i.log)"
  done
done
exit 0
