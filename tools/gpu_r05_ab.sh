#!/bin/bash
# Round 5 session AB: a second random-case soak on the final library -- 24x the suite's counts on
# another seed range (9,362 cases against the oracle).
S=tools/gpu_step.sh
TAIL=4 bash $S r05ab_random_soak 1100 env FLAME_RANDOM_SCALE=24 FLAME_RANDOM_SEED_OFFSET=2000000 python -u -m pytest tests/test_gpu_random_cases.py -x -q --timeout 300 --timeout-method thread
