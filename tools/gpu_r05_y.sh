#!/bin/bash
# Round 5 session Y: config 2 (256 clients x 1M fp32, 977 chunks, tiled slab) -- residency and
# client-unroll variants of its full-residency launch against the shipped kernel, one process.
S=tools/gpu_step.sh
V=flame_amd/libflame_amd.so:tiled,c2_lo:tiled,c2_lo_occ3:tiled,c2_lo_occ4:tiled,c2_cu4:tiled,c2_cu16:tiled
TAIL=8 bash $S r05y_c2_sweep 400 python3 tools/kernel_sweep.py --clients 256 --params 1004099 --rounds 8 --reps 10 --variants $V --out gpurun_out/r05y_c2.json
