#!/bin/bash
# Round 5 session V: the eager FedAvg round (64 x 25M fp32, one launch) through the kernel-argument
# metadata (default) and through the device table (FLAME_AMD_ARGMETA=0), twice each.
S=tools/gpu_step.sh
for i in 1 2; do
  TAIL=1 bash $S r05v_eager_argmeta_$i 300 python3 bench.py --workload fedavg_eager --steps 20 --warmup 3 --cpu-clients 0 &&
  TAIL=1 bash $S r05v_eager_table_$i 300 env FLAME_AMD_ARGMETA=0 python3 bench.py --workload fedavg_eager --steps 20 --warmup 3 --cpu-clients 0 || exit 1
done
