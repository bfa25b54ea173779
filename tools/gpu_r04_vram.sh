#!/bin/bash
# How long does a finished 100 GB process's VRAM take to come back, and does the next process's
# speed track it?  bench, then free-VRAM samples for 60 s in a separate process, then bench again.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04vr; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1
summ() { grep '^{' $OUT/$1.log | python -c "import json,sys; b=json.loads(sys.stdin.read()); r=b['roofline']; print('$1', round(b['ms_per_step'],3), round(r['kernel_ms'],3), round(r['measured_read_ceiling_GBps']), round(r['frac_of_measured_ceiling'],4))"; }
timeout -k 10 60 python tools/vram_state.py > $OUT/vram0.log 2>&1; tail -1 $OUT/vram0.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-clients 0 > $OUT/bench_1.log 2>&1 || exit 1
summ bench_1
timeout -k 10 120 python -u tools/vram_state.py --secs 60 --every 3 > $OUT/vram1.log 2>&1 || exit 1
grep -v amdgpu.ids $OUT/vram1.log | head -30
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-clients 0 > $OUT/bench_2.log 2>&1 || exit 1
summ bench_2
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-clients 0 > $OUT/bench_3.log 2>&1 || exit 1
summ bench_3
