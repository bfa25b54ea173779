#!/bin/bash
# Round 5 session E: the chain with the lane-aggregated admission check (4 compares per lane
# instead of 6 per element); FedOPT tests, chain A/B (round 4 / session C / now), the eager
# FedOPT bench lines.
S=tools/gpu_step.sh
TAIL=4 bash $S pytest_fedopt 600 python -u -m pytest tests -m gpu -x -q -k "chain or fedopt or fedadam or fedyogi or fedadagrad or admission" --timeout 300 --timeout-method thread &&
TAIL=12 bash $S chain_ab 300 python3 tools/chain_sweep.py --libs build/diag/lib_r04.so,build/diag/lib_r05c.so,flame_amd/libflame_amd.so --rounds 6 &&
TAIL=1 bash $S bench_fedadam_eager 300 python3 bench.py --workload fedadam_eager --steps 10 --warmup 2 &&
TAIL=1 bash $S bench_fedyogi_eager 300 python3 bench.py --workload fedyogi_eager --steps 10 --warmup 2 &&
TAIL=1 bash $S bench_fedadagrad_eager 300 python3 bench.py --workload fedadagrad_eager --steps 10 --warmup 2
