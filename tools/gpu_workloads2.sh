#!/bin/bash
# Re-measure C2 / C4 / eager end-to-end on the current kernels.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
for w in ${WORKLOADS:-c2 fedadam fedyogi fedadagrad e2e_copy e2e_eager}; do
  case $w in
    c2) W="--clients 256 --params 1000000 --seed 1 --steps 50 --warmup 5";;
    e2e_*) W="--e2e --e2e-mode ${w#e2e_} --steps 3 --warmup 1";;
    *) W="--workload $w";;
  esac
  timeout -k 10 300 python bench.py --cpu-clients 0 $W > $OUT/wl2_$w.log 2>&1
  rc=$?; echo "$w rc=$rc"; tail -1 $OUT/wl2_$w.log | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
done
