#!/bin/bash
# Round 5 session W: the fp32 chain with 2 / 3 / 4 chunks per workgroup and their outputs burst
# from LDS (FLAME_T_CHAIN_WGC) against the shipped chain, one process, bitwise; chain tests.
S=tools/gpu_step.sh
V=build/diag/variants
TAIL=4 bash $S r05w_pytest_chain 600 python -u -m pytest tests -m gpu -x -q -k "chain or eager or admission" --timeout 300 --timeout-method thread &&
TAIL=8 bash $S r05w_chain_wgc_ab 600 python3 tools/chain_sweep.py --rounds 6 \
  --libs flame_amd/libflame_amd.so,$V/lib_chain_wgc2.so,$V/lib_chain_wgc3.so,$V/lib_chain_wgc4_occ2.so
