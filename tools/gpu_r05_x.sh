#!/bin/bash
# Round 5 session X: the one-middle low-residency hierarchy launch (the async FedBuff top's fused
# scale_add) with 4 / 8 / 16 chunks per workgroup and the new weights burst from LDS
# (FLAME_T_HLO_WGC) against the shipped launch, one process, bitwise; fp32 and bf16, with and
# without the middle's delta; then the hierarchy / FedBuff GPU tests on the rebuilt library.
S=tools/gpu_step.sh
V=flame_amd/libflame_amd.so,hlo_wgc4,hlo_wgc8,hlo_wgc16
TAIL=6 bash $S r05x_fb_f32 400 python3 tools/fedbuff_sweep.py --variants $V --rounds 6 &&
TAIL=6 bash $S r05x_fb_bf16 400 python3 tools/fedbuff_sweep.py --variants $V --rounds 6 --dtype bf16 &&
TAIL=6 bash $S r05x_fb_f32_delta 400 python3 tools/fedbuff_sweep.py --variants $V --rounds 6 --delta &&
TAIL=4 bash $S r05x_pytest_hier 700 python -u -m pytest tests -m gpu -x -q -k "hier or fedbuff or low_residency or c5" --timeout 300 --timeout-method thread
