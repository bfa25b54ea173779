#!/bin/bash
# Round 5 session H: the fp32 chain at 16 loads per lane / 3 workgroups per CU (new default) vs
# round 4's library and configuration; the fast-path bit check and the FedOPT tests on this build.
S=tools/gpu_step.sh
V=build/diag/variants
TAIL=8 bash $S fp_probe 200 python3 tools/fp_probe.py --div-pairs 274877906944 &&
TAIL=4 bash $S pytest_fedopt 600 python -u -m pytest tests -m gpu -x -q -k "chain or fedopt or fedadam or fedyogi or fedadagrad or admission" --timeout 300 --timeout-method thread &&
TAIL=10 bash $S chain_ab 400 python3 tools/chain_sweep.py --libs build/diag/lib_r04.so,$V/lib_chain_cu8_full.so,flame_amd/libflame_amd.so --rounds 8
