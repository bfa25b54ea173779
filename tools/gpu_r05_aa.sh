#!/bin/bash
# Round 5 session AA: the bf16 eager FedOPT chain (64 x 25M bf16) -- residency and loads-in-flight
# variants against the shipped full-residency, 8-load chain, one process, bitwise.
S=tools/gpu_step.sh
V=build/diag/variants
TAIL=8 bash $S r05aa_chain16_ab 600 python3 tools/chain_sweep.py --dtype bf16 --rounds 6 \
  --libs flame_amd/libflame_amd.so,$V/lib_chain16_occ3.so,$V/lib_chain16_occ4.so,$V/lib_chain16_occ3_cu16.so,$V/lib_chain16_cu16.so,$V/lib_chain16_cu4.so
