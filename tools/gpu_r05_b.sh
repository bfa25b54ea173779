#!/bin/bash
# Round 5 session B: the fp32 sqrt / divide fast paths (exhaustive + randomized bit checks), the
# FedOPT GPU tests and the chain A/B against round 4's library; the wave-specialized hierarchy
# (FLAME_T_HIER_WS) through the hierarchy tests, A/B against the shipped build and its stamps;
# the CPU baseline's thread scaling.
S=tools/gpu_step.sh
TAIL=30 bash $S fp_probe 200 python3 tools/fp_probe.py --div-pairs 274877906944 &&
TAIL=4 bash $S pytest_fedopt 600 python -u -m pytest tests -m gpu -x -q -k "chain or fedopt or fedadam or fedyogi or fedadagrad or random or c4 or admission" --timeout 300 --timeout-method thread &&
TAIL=12 bash $S chain_ab 300 python3 tools/chain_sweep.py --libs build/diag/lib_r04.so,flame_amd/libflame_amd.so --rounds 6 &&
TAIL=4 bash $S pytest_hier_ws 400 env FLAME_AMD_LIB=build/diag/hier/lib_ws.so python -u -m pytest tests -m gpu -x -q -k "hier or c5 or sharded_hierarchy" --timeout 300 --timeout-method thread &&
TAIL=12 bash $S hier_ab 300 python3 tools/hier_sweep.py --variants flame_amd/libflame_amd.so,build/diag/hier/lib_ws.so --rounds 5 --mid-layout tiled &&
TAIL=30 bash $S hier_attrib_ws 300 python3 tools/hier_attrib.py --variant ws --out gpurun_out/r05_hier_attrib_ws.json &&
TAIL=8 bash $S cpu_scaling 300 python3 tools/cpu_baseline_scaling.py
