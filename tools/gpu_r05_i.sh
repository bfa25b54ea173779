#!/bin/bash
# Round 5 session I: the per-lane fast/slow select in adapt_vec (no ballot); FedOPT tests; chain
# A/B against round 4 and session H.
S=tools/gpu_step.sh
TAIL=4 bash $S pytest_fedopt 600 python -u -m pytest tests -m gpu -x -q -k "chain or fedopt or fedadam or fedyogi or fedadagrad or admission" --timeout 300 --timeout-method thread &&
TAIL=10 bash $S chain_ab 400 python3 tools/chain_sweep.py --libs build/diag/lib_r04.so,build/diag/lib_r05h.so,flame_amd/libflame_amd.so --rounds 8
