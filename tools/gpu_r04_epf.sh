#!/bin/bash
# Epilogue operand prefetch (FedOPT's cur / m / v, FedBuff's scale_add weights loaded ahead of
# the client stream): the previous product build vs the new one, same process, bitwise-checked.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04epf; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1
run() { local tag=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $OUT/$tag.log 2>&1; local rc=$?; echo "$tag rc=$rc"; grep -v amdgpu.ids $OUT/$tag.log | tail -${TAIL:-3} | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
A=build/diag/lib_prev.so; B=build/diag/lib_epf.so
run fedbuff_f32 300 python -u tools/fedbuff_sweep.py --variants $A,$B --rounds 8 --persistent-model
run fedbuff_bf16 300 python -u tools/fedbuff_sweep.py --variants $A,$B --rounds 8 --persistent-model --dtype bf16
TAIL=4 run fedadam 400 python -u tools/kernel_sweep.py --kernel fedadam --rounds 5 --variants $A:tiled,$B:tiled
TAIL=4 run fedyogi 400 python -u tools/kernel_sweep.py --kernel fedyogi --rounds 5 --variants $A:tiled,$B:tiled
TAIL=5 run hier 400 python -u tools/hier_sweep.py --mid-layout tiled --rounds 5 --variants $A,$B
