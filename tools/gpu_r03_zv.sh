#!/bin/bash
# The async FedBuff top aggregator's round (64 arrivals + fused scale_add: the single-middle hierarchy
# launch, full residency today) at 2 / 3 workgroups per CU, fp32 and bf16, bitwise across variants.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03zv; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 400 python -u tools/fedbuff_sweep.py --variants base,hocc2cu3,hocc2cu4,hocc3cu3 --rounds 5 \
  > $OUT/fedbuff_f32.log 2>&1 || { tail -20 $OUT/fedbuff_f32.log; exit 1; }
tail -6 $OUT/fedbuff_f32.log
timeout -k 10 400 python -u tools/fedbuff_sweep.py --variants base,hocc2cu3,hocc2cu4,hocc3cu3 --rounds 5 --dtype bf16 \
  > $OUT/fedbuff_bf16.log 2>&1 || { tail -20 $OUT/fedbuff_bf16.log; exit 1; }
tail -6 $OUT/fedbuff_bf16.log
