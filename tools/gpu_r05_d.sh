#!/bin/bash
# Round 5 session D: the wave-specialized hierarchy with dynamic LDS (112 VGPRs: two 5-wave
# workgroups per CU) vs the shipped build, its tests and stamps.
S=tools/gpu_step.sh
TAIL=12 bash $S hier_ab 400 python3 tools/hier_sweep.py --variants flame_amd/libflame_amd.so,build/diag/hier/lib_ws.so,build/diag/hier/lib_ws_hbl12.so,build/diag/hier/lib_ws_hbl12cu8.so --rounds 5 --mid-layout tiled &&
TAIL=30 bash $S hier_attrib_ws 300 python3 tools/hier_attrib.py --variant ws --out gpurun_out/r05d_hier_attrib_ws.json &&
TAIL=4 bash $S pytest_hier_ws 400 env FLAME_AMD_LIB=build/diag/hier/lib_ws.so python -u -m pytest tests -m gpu -x -q -k "hier or c5 or sharded_hierarchy" --timeout 300 --timeout-method thread
