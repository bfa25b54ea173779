#!/bin/bash
# Round 3: flame_agg_reduce's low-occupancy path (2 workgroups per CU, unroll 3) in the product:
# sweeps around it (fp32 and bf16), hierarchy / FedOPT residency variants, then the whole GPU
# suite and the default bench with the new library.  Needs build/variants and build/hvariants.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03zf; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
step() {
  local tag=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc"; tail -${TAIL:-1} $OUT/$tag.log | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
  return 0
}
TAIL=10 step hier_sweep 500 python -u tools/hier_sweep.py --rounds 3 --reps 3 --mid-layout tiled \
  --variants base,tailbcu3,tailbcu2,hcu3,lds12cu3,lds12cu4,lds8cu3,lds8cu2,rprobe
TAIL=7 step c3_sweep 500 python -u tools/kernel_sweep.py --rounds 3 --reps 3 --out $OUT/c3_sweep.json \
  --variants base:tiled,lo0:tiled,lo4:tiled,lo2occ3:tiled,lo3occ3:tiled,rprobe
TAIL=5 step c3_bf16_sweep 500 python -u tools/kernel_sweep.py --dtype bf16 --rounds 3 --reps 3 --out $OUT/c3_bf16_sweep.json \
  --variants base:tiled,lo0:tiled,lo4:tiled,rprobe
TAIL=5 step c4_sweep 500 python -u tools/kernel_sweep.py --kernel fedadam --rounds 3 --reps 3 --out $OUT/c4_sweep.json \
  --variants base:tiled,optwgc4cu3:tiled,optwgc4cu4:tiled,rprobe
TAIL=3 step pytest_gpu 900 python -u -m pytest tests -m gpu -q -x --timeout 600 --timeout-method thread
step bench_default 600 python bench.py
exit 0
