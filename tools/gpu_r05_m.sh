#!/bin/bash
# Round 5 session M: admission without the +-0 case for eta*m (float min/max of |num|, 9 instead of
# 13 VALU per 4-element step) against the shipped chain, one process, bitwise.
S=tools/gpu_step.sh
TAIL=6 bash $S r05m_chain_ab 500 python3 tools/chain_sweep.py --rounds 8 \
  --libs flame_amd/libflame_amd.so,build/diag/lib_nzero.so
