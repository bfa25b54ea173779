#!/bin/bash
# How long is the slow window after a process holding G GB exits?  For G = 100 and 250: a
# process allocates and fills G GB and exits; the next one probes an 8 GB buffer every 0.25 s.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04tr; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1
for G in 100 250; do
  timeout -k 10 120 python -c "import torch; x = torch.empty(int($G * 1e9) // 4, device='cuda'); x.fill_(1.0); torch.cuda.synchronize(); print('held', $G, 'GB')" || exit 1
  timeout -k 10 120 python -u tools/settle_probe.py --gb 8 --secs 12 --every 0.25 > $OUT/after_$G.log 2>&1 || exit 1
  echo "after $G GB:"; grep -v amdgpu.ids $OUT/after_$G.log | grep -v '^{' | tr '\n' ' ' | sed 's/GB\/s/|/g' | cut -c1-1500; echo
done
