#!/bin/bash
# Round 5 session T: where the LDS-held output bursts stop paying -- the low-residency reduction
# without bursts (lo_wgc1), with 8 / 16 chunks per workgroup at every client count, and the
# shipped choice (8 below 256 clients), fp32 at 64 / 128 / 256 / 512 clients and bf16 at 64 / 256.
S=tools/gpu_step.sh
V=lo_wgc1:tiled,flame_amd/libflame_amd.so:tiled,lo_wgc8_all:tiled,lo_wgc16_all:tiled
for n in 64 128 256 512; do
  TAIL=5 bash $S r05t_lo_wgc_$n 400 python3 tools/kernel_sweep.py --clients $n --rounds 5 --variants $V --out gpurun_out/r05t_$n.json || exit 1
done
for n in 64 256; do
  TAIL=5 bash $S r05t_lo_wgc_bf16_$n 400 python3 tools/kernel_sweep.py --dtype bf16 --clients $n --params 50000000 --rounds 5 --variants $V --out gpurun_out/r05t_bf16_$n.json || exit 1
done
