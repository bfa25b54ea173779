set -u
mkdir -p gpurun_out
export MASTER_ADDR=127.0.0.1
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541"
for f in 0.9,0.1 0.75,0.2,0.05 1.0 0.9,0.1; do
  timeout -k 10 400 $TR bench.py --force-shard --workload hier_fedbuff --steps 20 --warmup 5 --shard-fracs $f > gpurun_out/fr_$f.log 2>&1 || exit 1
  python -c "import json;d=json.loads([l for l in open('gpurun_out/fr_$f.log') if l.startswith('{')][-1]);print('$f', round(d['ms_per_step'],2), round(d['roofline']['kernel_ms'],2), round(d['host_issue_ms_per_step'],2))"
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_shard.py -x -q --timeout 200 --timeout-method thread 2>&1 | tail -2
