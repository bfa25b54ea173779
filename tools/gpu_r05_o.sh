#!/bin/bash
# Round 5 session O: the chain with EV chunks per lane (FLAME_T_CHAIN_EV: more independent step
# chains per lane) against the shipped chain, one process, bitwise; the chain / FedOPT tests on
# the rebuilt product library; then the random-case soak (12x the counts, fresh seeds).
S=tools/gpu_step.sh
V=build/diag/variants
TAIL=4 bash $S r05o_pytest_chain 600 python -u -m pytest tests -m gpu -x -q -k "chain or eager or admission" --timeout 300 --timeout-method thread &&
TAIL=10 bash $S r05o_chain_ev_ab 600 python3 tools/chain_sweep.py --rounds 6 \
  --libs flame_amd/libflame_amd.so,$V/lib_chain_ev2_cu8.so,$V/lib_chain_ev2_cu4.so,$V/lib_chain_ev2_cu8_occ2.so,$V/lib_chain_ev2_cu4_occ4.so,$V/lib_chain_ev4_cu4.so &&
TAIL=4 bash $S r05o_random_soak 900 env FLAME_RANDOM_SCALE=12 FLAME_RANDOM_SEED_OFFSET=1000000 python -u -m pytest tests/test_gpu_random_cases.py -x -q --timeout 300 --timeout-method thread
