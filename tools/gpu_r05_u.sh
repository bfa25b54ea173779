#!/bin/bash
# Round 5 session U: the low-residency reduction's LDS-held output bursts (below 512 clients)
# shipped: the whole GPU suite (new low-residency cases at 64 / 256 / 512 clients, the launch
# branch guard), smoke, the eager FedAvg round and the default bench.
S=tools/gpu_step.sh
TAIL=6 bash $S r05u_pytest_gpu 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations 5 &&
TAIL=2 bash $S r05u_smoke 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" &&
TAIL=1 bash $S r05u_bench_fedavg_eager 300 python3 bench.py --workload fedavg_eager --steps 10 --warmup 3 --cpu-clients 0 &&
TAIL=1 bash $S r05u_bench_default 300 python3 bench.py
