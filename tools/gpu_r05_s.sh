#!/bin/bash
# Round 5 session S: the low-residency reduction with G chunks per workgroup and their outputs
# held in LDS, stored in one burst (FLAME_T_LO_WGC) -- the 64-client eager FedAvg round's shape and
# C3's -- against the shipped kernel, tiled slab, one process per client count, bitwise-checked.
S=tools/gpu_step.sh
V=flame_amd/libflame_amd.so:tiled,lo_wgc8:tiled,lo_wgc16:tiled,lo_wgc32:tiled,lo_wgc16_1cu:tiled
TAIL=8 bash $S r05s_lo_wgc_64 400 python3 tools/kernel_sweep.py --clients 64 --rounds 5 --variants $V --out gpurun_out/r05s_64.json &&
TAIL=8 bash $S r05s_lo_wgc_1024 600 python3 tools/kernel_sweep.py --clients 1024 --rounds 3 --variants $V --out gpurun_out/r05s_1024.json
