#!/bin/bash
# Round 5 session C: the chain kernel with scalar step_end loads and a workgroup-uniform vector
# path (per-load waits instead of vmcnt(0)), A/B against round 4's library and session B's; the
# wave-specialized hierarchy with packed sums at 16 / 14 / 12-middle store groups vs the shipped
# build, its tests and stamps.
S=tools/gpu_step.sh
TAIL=4 bash $S pytest_fedopt 600 python -u -m pytest tests -m gpu -x -q -k "chain or fedopt or fedadam or fedyogi or fedadagrad or admission" --timeout 300 --timeout-method thread &&
TAIL=12 bash $S chain_ab 300 python3 tools/chain_sweep.py --libs build/diag/lib_r04.so,build/diag/lib_r05b.so,flame_amd/libflame_amd.so --rounds 6 &&
TAIL=12 bash $S hier_ab 400 python3 tools/hier_sweep.py --variants flame_amd/libflame_amd.so,build/diag/hier/lib_ws.so,build/diag/hier/lib_ws_hbl14.so,build/diag/hier/lib_ws_hbl12.so,build/diag/hier/lib_ws_hbl12cu8.so,build/diag/hier/lib_ws_hbl12cu4.so --rounds 5 --mid-layout tiled &&
TAIL=4 bash $S pytest_hier_ws 400 env FLAME_AMD_LIB=build/diag/hier/lib_ws_hbl12.so python -u -m pytest tests -m gpu -x -q -k "hier or c5 or sharded_hierarchy" --timeout 300 --timeout-method thread &&
TAIL=30 bash $S hier_attrib_ws 300 python3 tools/hier_attrib.py --variant ws --out gpurun_out/r05c_hier_attrib_ws.json
