#!/bin/bash
# Round 5 session Q: the random-case soak on the shipped library, and bench.py --gpus 8 with no
# launcher over gloo (8 ranks sharing the one GPU: the spawn path and the N = 8 layout).
S=tools/gpu_step.sh
TAIL=4 bash $S r05q_random_soak 900 env FLAME_RANDOM_SCALE=12 FLAME_RANDOM_SEED_OFFSET=1000000 python -u -m pytest tests/test_gpu_random_cases.py -x -q --timeout 300 --timeout-method thread &&
TAIL=1 bash $S r05q_gpus8_gloo 600 env FLAME_BENCH_BACKEND=gloo python3 bench.py --gpus 8 --clients 64 --params 2000000 --steps 5 --warmup 2
