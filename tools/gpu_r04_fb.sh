#!/bin/bash
# FedBuff top: bench.py's fedbuff line vs tools/fedbuff_sweep.py's same-process rounds, one box,
# bisecting why the bench's kernel (1.01-1.06 ms) is slower than the sweep's (0.97 ms).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04fb; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1
run() { local tag=$1; shift; timeout -k 10 300 "$@" > $OUT/$tag.log 2>&1; local rc=$?; echo "$tag rc=$rc"; grep -v amdgpu.ids $OUT/$tag.log | tail -3 | cut -c1-600; [ $rc -eq 0 ] || exit $rc; }
L=flame_amd/libflame_amd.so
run sweep python tools/fedbuff_sweep.py --variants $L --rounds 8
run sweep_synth python tools/fedbuff_sweep.py --variants $L --rounds 8 --stale synth
run sweep_persist python tools/fedbuff_sweep.py --variants $L --rounds 8 --persistent-model
run sweep_both python tools/fedbuff_sweep.py --variants $L --rounds 8 --stale synth --persistent-model
run bench python bench.py --workload fedbuff --steps 20 --warmup 3 --cpu-clients 0
