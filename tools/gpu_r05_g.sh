#!/bin/bash
# Round 5 session G: more chain unroll x residency variants (one process, bitwise-checked) and
# one SQ counter pass on the shipped chain kernel (its own run, no trace domains).
S=tools/gpu_step.sh
V=build/diag/variants
TAIL=14 bash $S chain_ab 500 python3 tools/chain_sweep.py --libs flame_amd/libflame_amd.so,$V/lib_chain_cu16.so,$V/lib_chain_occ3.so,$V/lib_chain_cu16_occ3.so,$V/lib_chain_cu16_occ4.so,$V/lib_chain_cu12_occ3.so,$V/lib_chain_cu32.so,$V/lib_chain_cu24_occ3.so,$V/lib_chain_occ2.so --rounds 6 &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
TAIL=3 bash $S chain_pmc_sq 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD --kernel-include-regex fedopt_chain --output-format csv -d gpurun_out/chain_pmc_sq -o run -- python3 bench.py --workload fedadam_eager --steps 3 --warmup 1 --cpu-clients 0
