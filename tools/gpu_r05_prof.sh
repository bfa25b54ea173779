#!/bin/bash
# Round 5 evidence session: for each default path, bench.py's line under
# `rocprofv3 --kernel-trace --stats` (the kernel-trace summary of the SAME process), then the PMC
# pairs (FETCH_SIZE, then WRITE_SIZE, each its own run, no trace domains) for the headline FedAvg,
# the eager FedOPT chain and config 5's hierarchy -> gpurun_out/r05prof/traffic.json
# (tools/pmc_traffic.py, gfx950 FETCH_SIZE x2 correction).  Archive with:
#   cp gpurun_out/r05prof/<w>.log profiles/r05prof_<w>.log; cp .../<w>/run_kernel_stats.csv ...
S=tools/gpu_step.sh
O=gpurun_out/r05prof
mkdir -p $O
export TMPDIR=/tmp
prof() {  # prof <tag> <bench args...>
  local tag=$1; shift
  TAIL=1 bash $S r05prof/$tag 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag -o run -- \
      python3 bench.py "$@" && rm -f $O/$tag/run_kernel_trace.csv
}
pmc() {  # pmc <tag> <kernel regex> <bench args...>
  local tag=$1 rx=$2; shift 2
  for C in FETCH_SIZE WRITE_SIZE; do
    TAIL=1 bash $S r05prof/pmc_${tag}_$C 120 rocprofv3 --pmc $C --kernel-include-regex $rx --output-format csv \
        -d $O/pmc_${tag}_$C -o run -- python3 bench.py "$@" --steps 3 --warmup 1 --cpu-clients 0 || return 1
  done
}
prof fedavg --steps 20 --warmup 5 &&
prof fedadam --workload fedadam --steps 10 --warmup 3 --cpu-clients 16 &&
prof fedyogi --workload fedyogi --steps 10 --warmup 3 --cpu-clients 0 &&
prof fedadagrad --workload fedadagrad --steps 10 --warmup 3 --cpu-clients 0 &&
prof hier_fedbuff --workload hier_fedbuff --steps 10 --warmup 3 --cpu-clients 0 &&
prof fedbuff --workload fedbuff --steps 10 --warmup 3 --cpu-clients 0 &&
prof fedadam_eager --workload fedadam_eager --steps 10 --warmup 3 --cpu-clients 0 &&
prof fedyogi_eager --workload fedyogi_eager --steps 10 --warmup 3 --cpu-clients 0 &&
prof fedadagrad_eager --workload fedadagrad_eager --steps 10 --warmup 3 --cpu-clients 0 &&
prof feddyn --workload feddyn --steps 6 --warmup 2 --cpu-clients 0 &&
pmc fedavg agg_reduce &&
pmc fedadam_eager fedopt_chain --workload fedadam_eager &&
pmc hier_fedbuff hier_fedbuff --workload hier_fedbuff &&
cp profiles/traffic.json $O/traffic.json &&
python3 tools/pmc_traffic.py --fetch $O/pmc_fedavg_FETCH_SIZE --write $O/pmc_fedavg_WRITE_SIZE --layout slab --workload fedavg \
    --source "profiles/r05prof_pmc_fedavg_{FETCH,WRITE}_SIZE.csv (round 5, tools/gpu_r05_prof.sh)" --out $O/traffic.json &&
python3 tools/pmc_traffic.py --fetch $O/pmc_fedadam_eager_FETCH_SIZE --write $O/pmc_fedadam_eager_WRITE_SIZE \
    --kernel fedopt_chain --name flame_fedopt_chain --clients 64 --extra-arrays 8 --layout slab --workload fedadam_eager \
    --source "profiles/r05prof_pmc_fedadam_eager_{FETCH,WRITE}_SIZE.csv (round 5, tools/gpu_r05_prof.sh)" --out $O/traffic.json &&
python3 tools/pmc_traffic.py --fetch $O/pmc_hier_fedbuff_FETCH_SIZE --write $O/pmc_hier_fedbuff_WRITE_SIZE \
    --kernel hier_fedbuff --name flame_hier_fedbuff --clients 4096 --params 15625000 --itemsize 2 --extra-arrays 131 \
    --layout slab --workload hier_fedbuff --source "profiles/r05prof_pmc_hier_fedbuff_{FETCH,WRITE}_SIZE.csv (round 5, tools/gpu_r05_prof.sh)" \
    --out $O/traffic.json
