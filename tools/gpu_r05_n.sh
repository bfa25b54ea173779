#!/bin/bash
# Round 5 session N: a soak of the randomised differential tests -- 12x the suite's case counts
# on fresh seeds (4,680 cases: FedAvg / FedBuff / FedOPT / eager, hierarchies, FedDyn /
# SCAFFOLD, 16-bit eager FedOPT), every one against the oracle.
S=tools/gpu_step.sh
TAIL=4 bash $S r05n_random_soak 1100 env FLAME_RANDOM_SCALE=12 FLAME_RANDOM_SEED_OFFSET=1000000 python -u -m pytest tests/test_gpu_random_cases.py -x -q --timeout 300 --timeout-method thread
