#!/bin/bash
# contiguous vs caching-allocator buffers, right after a large process exits and after 90 s
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04ct; mkdir -p $OUT
export PYTHONDONTWRITEBYTECODE=1
run() { local tag=$1; shift; timeout -k 10 300 "$@" > $OUT/$tag.log 2>&1; local rc=$?; echo "$tag rc=$rc"; grep -v amdgpu.ids $OUT/$tag.log | grep -v '^{' | head -4 | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
run bench python bench.py --steps 5 --warmup 2 --cpu-clients 0
run dirty python -u tools/contig_probe.py --order contig,torch
run dirty2 python -u tools/contig_probe.py --order torch,contig
echo "pause 90 s"; sleep 90
run settled python -u tools/contig_probe.py --order contig,torch
