#!/bin/bash
# Round 5 session J: v below 2^-96 admitted to the fast sqrt (no lower-bound reduction); the
# fp probe (incl. sqrt(v) + tau below 2^-96), FedOPT tests, chain A/B against round 4 and
# session I, then the eager bench lines.
S=tools/gpu_step.sh
TAIL=6 bash $S r05j_fp_probe 300 python3 tools/fp_probe.py &&
TAIL=4 bash $S r05j_pytest_fedopt 600 python -u -m pytest tests -m gpu -x -q -k "chain or fedopt or fedadam or fedyogi or fedadagrad or admission" --timeout 300 --timeout-method thread &&
TAIL=10 bash $S r05j_chain_ab 400 python3 tools/chain_sweep.py --libs build/diag/lib_r04.so,build/diag/lib_r05i.so,flame_amd/libflame_amd.so --rounds 8 &&
for w in fedadam_eager fedyogi_eager fedadagrad_eager; do
  TAIL=1 bash $S r05j_bench_$w 300 python3 bench.py --workload $w --steps 10 --warmup 3 --cpu-clients 0 || exit 1
done
