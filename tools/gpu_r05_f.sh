#!/bin/bash
# Round 5 session F: the chain with the batch's scalar loads issued together; client unroll and
# residency variants of it, one process, bitwise-checked.
S=tools/gpu_step.sh
TAIL=4 bash $S pytest_chain 400 python -u -m pytest tests -m gpu -x -q -k "chain or admission" --timeout 300 --timeout-method thread &&
TAIL=12 bash $S chain_ab 400 python3 tools/chain_sweep.py --libs build/diag/lib_r05c.so,flame_amd/libflame_amd.so,build/diag/variants/lib_chain_cu4.so,build/diag/variants/lib_chain_cu16.so,build/diag/variants/lib_chain_occ4.so,build/diag/variants/lib_chain_occ3.so --rounds 6
