set -u
mkdir -p gpurun_out
for h in rows pingpong pingpong_rows rows; do
  timeout -k 10 300 python bench.py --workload feddyn --steps 8 --warmup 2 --feddyn-history $h > gpurun_out/dyn_$h.log 2>&1 || exit 1
  python -c "import json;d=json.loads([l for l in open('gpurun_out/dyn_$h.log') if l.startswith('{')][-1]);print('$h', round(d['ms_per_step'],2), round(d['roofline']['kernel_ms_per_step'],2))"
done
timeout -k 10 300 python bench.py --workload feddyn --steps 8 --warmup 2 --feddyn-order shuffled --feddyn-history pingpong > gpurun_out/dyn_shuf_pp.log 2>&1 && tail -c 300 gpurun_out/dyn_shuf_pp.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "feddyn" -x -q --timeout 200 --timeout-method thread 2>&1 | tail -3
