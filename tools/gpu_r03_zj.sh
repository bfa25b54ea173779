#!/bin/bash
# SQ counters (one pass each, 8 SQ counters) on the hierarchy kernel and the C3 reduction: where a
# wave's time goes (VALU / VMEM / scalar / waiting) at the same residency.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03zj; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
PMC="SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_ANY SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_SCA"
timeout -s KILL 300 rocprofv3 --pmc $PMC --kernel-include-regex hier_fedbuff --output-format csv -d $OUT/sq_hier -o run -- \
  python bench.py --workload hier_fedbuff --steps 3 --warmup 1 --cpu-clients 0 > $OUT/sq_hier.log 2>&1 || { echo "hier rc=$?"; tail -3 $OUT/sq_hier.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc $PMC --kernel-include-regex agg_reduce --output-format csv -d $OUT/sq_c3 -o run -- \
  python bench.py --steps 3 --warmup 1 --cpu-clients 0 > $OUT/sq_c3.log 2>&1 || { echo "c3 rc=$?"; tail -3 $OUT/sq_c3.log; exit 1; }
PMC2="SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_INST_CYCLES_SMEM SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_LDS"
timeout -s KILL 300 rocprofv3 --pmc $PMC2 --kernel-include-regex hier_fedbuff --output-format csv -d $OUT/sq2_hier -o run -- \
  python bench.py --workload hier_fedbuff --steps 3 --warmup 1 --cpu-clients 0 > $OUT/sq2_hier.log 2>&1 || { echo "hier2 rc=$?"; tail -3 $OUT/sq2_hier.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc $PMC2 --kernel-include-regex agg_reduce --output-format csv -d $OUT/sq2_c3 -o run -- \
  python bench.py --steps 3 --warmup 1 --cpu-clients 0 > $OUT/sq2_c3.log 2>&1 || { echo "c32 rc=$?"; tail -3 $OUT/sq2_c3.log; exit 1; }
echo done
