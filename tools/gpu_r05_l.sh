#!/bin/bash
# Round 5 session L: the eager bench's chain against tools/chain_sweep.py's on one box (is the
# bench's ~4 % higher chain time the workload or the box?), and the shipped chain's SQ counters.
S=tools/gpu_step.sh
export TMPDIR=/tmp
TAIL=3 bash $S r05l_chain_sweep_1 300 python3 tools/chain_sweep.py --rounds 6 --libs flame_amd/libflame_amd.so &&
TAIL=1 bash $S r05l_bench_fedadam_eager 300 python3 bench.py --workload fedadam_eager --steps 10 --warmup 3 --cpu-clients 0 &&
TAIL=3 bash $S r05l_chain_sweep_2 300 python3 tools/chain_sweep.py --rounds 6 --libs flame_amd/libflame_amd.so &&
TAIL=1 bash $S r05l_bench_fedadam_eager_2 300 python3 bench.py --workload fedadam_eager --steps 10 --warmup 3 --cpu-clients 0 &&
TAIL=3 bash $S r05l_chain_pmc_sq 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD --kernel-include-regex fedopt_chain --output-format csv -d gpurun_out/r05l_chain_pmc_sq -o run -- python3 bench.py --workload fedadam_eager --steps 3 --warmup 1 --cpu-clients 0
