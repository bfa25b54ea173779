#!/bin/bash
# Round 5 evidence session: for each default path, bench.py's line under
# `rocprofv3 --kernel-trace --stats` (the kernel-trace summary of the SAME process), then the PMC
# pairs (FETCH_SIZE, then WRITE_SIZE, each its own run, no trace domains) for the headline FedAvg,
# the eager FedOPT chain and config 5's hierarchy -> gpurun_out/r05prof/traffic.json
# (tools/pmc_traffic.py, gfx950 FETCH_SIZE x2 correction).  Archive with:
#   cp gpurun_out/$T/<w>.log profiles/$T_<w>.log; cp .../<w>/run_kernel_stats.csv ...
# T (default r05prof) names the collection.
S=tools/gpu_step.sh
T=${T:-r05prof}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
prof() {  # prof <tag> <bench args...>
  local tag=$1; shift
  TAIL=1 bash $S $T/$tag 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag -o run -- \
      python3 bench.py "$@" && rm -f $O/$tag/run_kernel_trace.csv
}
pmc() {  # pmc <tag> <kernel regex> <bench args...>
  local tag=$1 rx=$2; shift 2
  for C in FETCH_SIZE WRITE_SIZE; do
    TAIL=1 bash $S $T/pmc_${tag}_$C 120 rocprofv3 --pmc $C --kernel-include-regex $rx --output-format csv \
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
b() {  # b <tag> <bench args...>: a plain bench line (no profiler)
  local tag=$1; shift
  TAIL=1 bash $S $T/bench_$tag 400 python3 bench.py --cpu-clients 0 "$@"
}
b c2 --clients 256 --params 1000000 --steps 50 --warmup 5 &&
b fedavg_eager --workload fedavg_eager --steps 10 --warmup 3 &&
b scaffold --workload scaffold --steps 10 --warmup 3 &&
b hier_fetched --workload hier_fedbuff --hier-middles fetched --steps 10 --warmup 3 &&
b hier_sync --workload hier_fedbuff --hier-mode sync --steps 10 --warmup 3 &&
pmc fedavg agg_reduce &&
pmc fedadam_eager fedopt_chain --workload fedadam_eager &&
pmc hier_fedbuff hier_fedbuff --workload hier_fedbuff &&
cp profiles/traffic.json $O/traffic.json &&
python3 tools/pmc_traffic.py --fetch $O/pmc_fedavg_FETCH_SIZE --write $O/pmc_fedavg_WRITE_SIZE --layout slab --workload fedavg \
    --source "profiles/${T}_pmc_fedavg_{FETCH,WRITE}_SIZE.csv (round 5, tools/gpu_r05_prof.sh)" --out $O/traffic.json &&
python3 tools/pmc_traffic.py --fetch $O/pmc_fedadam_eager_FETCH_SIZE --write $O/pmc_fedadam_eager_WRITE_SIZE \
    --kernel fedopt_chain --name flame_fedopt_chain --clients 64 --extra-arrays 8 --layout slab --workload fedadam_eager \
    --source "profiles/${T}_pmc_fedadam_eager_{FETCH,WRITE}_SIZE.csv (round 5, tools/gpu_r05_prof.sh)" --out $O/traffic.json &&
python3 tools/pmc_traffic.py --fetch $O/pmc_hier_fedbuff_FETCH_SIZE --write $O/pmc_hier_fedbuff_WRITE_SIZE \
    --kernel hier_fedbuff --name flame_hier_fedbuff --clients 4096 --params 15625000 --itemsize 2 --extra-arrays 131 \
    --layout slab --workload hier_fedbuff --source "profiles/${T}_pmc_hier_fedbuff_{FETCH,WRITE}_SIZE.csv (round 5, tools/gpu_r05_prof.sh)" \
    --out $O/traffic.json
