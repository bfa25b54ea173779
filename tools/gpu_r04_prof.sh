#!/bin/bash
# Round 4 evidence for the shipped build, per default path: the bench line and the rocprofv3
# kernel-trace summary of the SAME process, then the PMC pair (FETCH_SIZE / WRITE_SIZE, one
# counter per run, no trace domains) -> profiles/traffic.json entries.
#   PART=A: C3, C4 FedAdam, C4 FedYogi     PART=B: C4 FedAdaGrad, C5 shard, async FedBuff top
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04prof; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
step() {
  local tag=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc"; grep '^{' $OUT/$tag.log | cut -c1-200
  if [ $rc -ne 0 ]; then tail -5 $OUT/$tag.log; exit $rc; fi
  return 0
}
cp profiles/traffic.json $OUT/traffic.json
# prof <tag> <kernel regex> <report name> <clients> <params> <itemsize> <extra arrays> <bench args...>
prof() {
  local tag=$1 rx=$2 name=$3 cl=$4 pa=$5 isz=$6 extra=$7; shift 7
  step prof_$tag 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$tag -o run -- \
      python bench.py --cpu-clients 0 "$@"
  rm -f $OUT/prof_$tag/run_kernel_trace.csv
  for C in FETCH_SIZE WRITE_SIZE; do
    step pmc_${tag}_$C 600 rocprofv3 --pmc $C --kernel-include-regex $rx --output-format csv \
        -d $OUT/pmc_${tag}_$C -o run -- python bench.py --cpu-clients 0 "$@" --steps 3 --warmup 1
  done
  python tools/pmc_traffic.py --fetch $OUT/pmc_${tag}_FETCH_SIZE --write $OUT/pmc_${tag}_WRITE_SIZE --kernel $rx \
      --name $name --clients $cl --params $pa --itemsize $isz --extra-arrays $extra --layout slab --workload $tag \
      --out $OUT/traffic.json | cut -c1-300
}
if [ "${PART:-A}" = A ]; then
  prof fedavg agg_reduce flame_agg_reduce 1024 25000000 4 2 --steps 10 --warmup 3
  prof fedadam fedopt_kernel flame_fedopt_reduce_adapt 1024 25000000 4 8 --workload fedadam --steps 10 --warmup 3
  prof fedyogi fedopt_kernel flame_fedopt_reduce_adapt 1024 25000000 4 8 --workload fedyogi --steps 10 --warmup 3
elif [ "${PART:-A}" = C ]; then
  # the other shipped paths' bench lines (kernels unchanged this round; re-measured on this build)
  step bench_c2 300 python bench.py --clients 256 --params 1000000 --steps 50 --warmup 5 --cpu-clients 0
  step bench_eager 300 python bench.py --workload fedavg_eager --steps 10 --warmup 3 --cpu-clients 0
  step bench_fedadam_eager 300 python bench.py --workload fedadam_eager --steps 5 --warmup 2
  step bench_scaffold 400 python bench.py --workload scaffold --steps 10 --warmup 3 --cpu-clients 0
  step bench_feddyn 400 python bench.py --workload feddyn --steps 8 --warmup 2
  step bench_hier_fetched 400 python bench.py --workload hier_fedbuff --hier-middles fetched --steps 10 --warmup 3 --cpu-clients 0
  step bench_hier_sync 400 python bench.py --workload hier_fedbuff --hier-mode sync --steps 10 --warmup 3 --cpu-clients 0
else
  prof fedadagrad fedopt_kernel flame_fedopt_reduce_adapt 1024 25000000 4 8 --workload fedadagrad --steps 10 --warmup 3
  prof hier_fedbuff hier_fedbuff flame_hier_fedbuff 4096 15625000 2 131 --workload hier_fedbuff --steps 10 --warmup 3
  prof fedbuff hier_fedbuff flame_hier_fedbuff 64 25000000 4 2 --workload fedbuff --steps 10 --warmup 3
fi
exit 0
