#!/bin/bash
# Cross-process spread of the default bench line: the same command in 4 fresh processes on one
# box, each with its own same-process read probes ("Cross-process spread").
# SETTLE=0: bench.py's settle step off (FLAME_BENCH_SETTLE=0), as before it existed.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04sp${TAG:-}; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 FLAME_BENCH_SETTLE=${SETTLE:-1}
for i in 1 2 3 4; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-clients 0 > $OUT/bench_$i.log 2>&1
  rc=$?; echo "run $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  grep '^{' $OUT/bench_$i.log | python -c "import json,sys; b=json.loads(sys.stdin.read()); r=b['roofline']; st=b.get('settle') or {}; print(round(b['ms_per_step'],3), round(r['kernel_ms'],3), round(r['frac'],4), round(r['measured_read_ceiling_GBps']), round(r['frac_of_measured_ceiling'],4), 'settle', st.get('waited_s'), st.get('probe_GBps'))"
done
