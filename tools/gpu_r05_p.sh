#!/bin/bash
# Round 5 session P: C4's fused FedOPT kernel, round 4's library vs the shipped one (fast sqrt /
# divide in the epilogue) in one process, per variant: is the 1-3 % between FedAdam / FedAdaGrad
# and FedYogi in the bench lines the library or the process?
S=tools/gpu_step.sh
for k in fedadam fedyogi fedadagrad; do
  TAIL=6 bash $S r05p_c4_ab_$k 400 python3 tools/kernel_sweep.py --kernel $k --rounds 5 \
    --variants build/diag/lib_r04.so,flame_amd/libflame_amd.so,build/diag/lib_r04.so,flame_amd/libflame_amd.so --out gpurun_out/r05p_$k.json || exit 1
done
