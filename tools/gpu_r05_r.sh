#!/bin/bash
# Round 5 session R: PMC traffic (FETCH_SIZE, then WRITE_SIZE, separate runs) for the secondary
# paths' bench lines -- FedDyn, the eager FedAvg round, C2, C5 with fetched middles -- appended to
# a copy of profiles/traffic.json (gpurun_out/r05r/traffic.json).
S=tools/gpu_step.sh
O=gpurun_out/r05r
mkdir -p $O
export TMPDIR=/tmp
pmc() {  # pmc <tag> <kernel regex> <bench args...>
  local tag=$1 rx=$2; shift 2
  for C in FETCH_SIZE WRITE_SIZE; do
    TAIL=1 bash $S r05r/pmc_${tag}_$C 300 rocprofv3 --pmc $C --kernel-include-regex $rx --output-format csv \
        -d $O/pmc_${tag}_$C -o run -- python3 bench.py "$@" --steps 3 --warmup 1 --cpu-clients 0 || return 1
  done
}
src() { echo "profiles/r05r_pmc_$1_{FETCH,WRITE}_SIZE.csv (round 5, tools/gpu_r05_r.sh)"; }
pmc feddyn feddyn --workload feddyn &&
pmc fedavg_eager agg_reduce --workload fedavg_eager &&
pmc c2 agg_reduce --clients 256 --params 1000000 &&
pmc hier_fetched hier_fedbuff --workload hier_fedbuff --hier-middles fetched &&
cp profiles/traffic.json $O/traffic.json &&
python3 tools/pmc_traffic.py --fetch $O/pmc_feddyn_FETCH_SIZE --write $O/pmc_feddyn_WRITE_SIZE --kernel feddyn \
    --name flame_feddyn_round --clients 512 --extra-arrays 1027 --workload feddyn --source "$(src feddyn)" --out $O/traffic.json &&
python3 tools/pmc_traffic.py --fetch $O/pmc_fedavg_eager_FETCH_SIZE --write $O/pmc_fedavg_eager_WRITE_SIZE --kernel agg_reduce \
    --name flame_agg_reduce --clients 64 --extra-arrays 2 --workload fedavg_eager --source "$(src fedavg_eager)" --out $O/traffic.json &&
python3 tools/pmc_traffic.py --fetch $O/pmc_c2_FETCH_SIZE --write $O/pmc_c2_WRITE_SIZE --kernel agg_reduce \
    --name flame_agg_reduce --clients 256 --params 1000000 --extra-arrays 2 --workload fedavg --source "$(src c2)" --out $O/traffic.json &&
python3 tools/pmc_traffic.py --fetch $O/pmc_hier_fetched_FETCH_SIZE --write $O/pmc_hier_fetched_WRITE_SIZE --kernel hier_fedbuff \
    --name flame_hier_fedbuff --clients 4096 --params 15625000 --itemsize 2 --extra-arrays 4 --workload hier_fedbuff_fetched \
    --source "$(src hier_fetched)" --out $O/traffic.json
