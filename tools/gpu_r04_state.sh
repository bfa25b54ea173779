#!/bin/bash
# Cross-process spread, continued: the state probe in one process (allocation vs streaming
# time), then the default bench twice back to back, a 120 s pause, and once more.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04st; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1
run() { local tag=$1; shift; timeout -k 10 300 "$@" > $OUT/$tag.log 2>&1; local rc=$?; echo "$tag rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
summ() { grep '^{' $OUT/$1.log | python -c "import json,sys; b=json.loads(sys.stdin.read()); r=b['roofline']; print('$1', round(b['ms_per_step'],3), round(r['kernel_ms'],3), round(r['measured_read_ceiling_GBps']), round(r['frac_of_measured_ceiling'],4))"; }
run state python -u tools/state_probe.py --heat 40
grep -v amdgpu.ids $OUT/state.log | head -4 | cut -c1-200
run bench_a python bench.py --steps 10 --warmup 3 --cpu-clients 0 && summ bench_a
run bench_b python bench.py --steps 10 --warmup 3 --cpu-clients 0 && summ bench_b
echo "pause 120 s"; sleep 120
run bench_c python bench.py --steps 10 --warmup 3 --cpu-clients 0 && summ bench_c
