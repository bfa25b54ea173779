#!/bin/bash
# Round 5 session K: software-pipelined chain batches (FLAME_T_CHAIN_PIPE) against the shipped
# chain, one process, bitwise-checked.
S=tools/gpu_step.sh
V=build/diag/variants
TAIL=10 bash $S r05k_chain_ab 500 python3 tools/chain_sweep.py --rounds 6 \
  --libs flame_amd/libflame_amd.so,$V/lib_chain_pipe8.so,$V/lib_chain_pipe12.so,$V/lib_chain_pipe16.so,$V/lib_chain_pipe8_occ4.so,$V/lib_chain_pipe4_occ4.so
