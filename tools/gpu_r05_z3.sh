#!/bin/bash
# Round 5 closing session (3) on the final tree: the whole GPU suite (with the oracle-only launch
# branch guard last), smoke(), the default bench line, and the --gpus 2 path over gloo.
S=tools/gpu_step.sh
TAIL=6 bash $S r05z3_pytest_gpu 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations 5 &&
TAIL=3 bash $S r05z3_smoke 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" &&
TAIL=1 bash $S r05z3_bench_default 300 python3 bench.py &&
TAIL=1 bash $S r05z3_gpus2_gloo 400 env FLAME_BENCH_BACKEND=gloo python3 bench.py --gpus 2 --clients 64 --params 2000000
