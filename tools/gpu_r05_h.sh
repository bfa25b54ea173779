#!/bin/bash
# Round 5 session H: the fp32 chain at 16 loads per lane / 3 workgroups per CU (new default) vs
# round 4's configuration and the seed-nudge sqrt variant; the nudge's bit check; the FedOPT tests.
S=tools/gpu_step.sh
V=build/diag/variants
TAIL=8 bash $S fp_probe_nudge 200 python3 tools/fp_probe.py --lib build/diag/libfp_probe_nudge.so --div-pairs 1e9 &&
TAIL=4 bash $S pytest_fedopt 600 python -u -m pytest tests -m gpu -x -q -k "chain or fedopt or fedadam or fedyogi or fedadagrad or admission" --timeout 300 --timeout-method thread &&
TAIL=10 bash $S chain_ab 400 python3 tools/chain_sweep.py --libs build/diag/lib_r04.so,$V/lib_chain_cu8_full.so,flame_amd/libflame_amd.so,$V/lib_sqrt_nudge.so --rounds 8
