#!/bin/bash
# Hierarchy kernel with LDS-held store groups (FLAME_HLDS) vs the register groups it replaced
# (variant "nolds"), config 5 shard, every middle layout / mode / dtype; then the product
# library's bench + kernel trace.  Needs build/hvariants (drop it from .gpurunignore for the call).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
fatal() { rc=$1; [ "$rc" -ge 124 ] || [ "$rc" -gt 128 ]; }
step() {  # step <tag> <timeout> <cmd...>
  local tag=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc"; tail -${TAIL:-1} $OUT/$tag.log | cut -c1-300
  if fatal $rc || [ $rc -ne 0 ]; then exit $rc; fi
  return 0
}
TAIL=6 step hlds_bf16 400 python -u tools/hier_sweep.py --variants base:tiled,nolds:tiled,base,nolds,base:sync,nolds:sync,hdiag1:tiled --rounds 4
TAIL=6 step hlds_f32 400 python -u tools/hier_sweep.py --dtype f32 --params 7812500 --variants base:tiled,nolds:tiled,base,nolds,base:sync,nolds:sync --rounds 4
TAIL=3 step hlds_pytest 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -k "hier or fedbuff or FedBuff or c5 or shard or golden"
TAIL=2 step hlds_bench 400 python bench.py --workload hier_fedbuff --steps 10 --warmup 3 --cpu-clients 0
TAIL=2 step hlds_bench_sync 400 python bench.py --workload hier_fedbuff --hier-mode sync --steps 10 --warmup 3 --cpu-clients 0
cd /tmp && export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/$OUT/prof_hlds" -o run -- python3 "$R/bench.py" --workload hier_fedbuff --steps 10 --warmup 3 --cpu-clients 0 > "$R/$OUT/hlds_bench_prof.log" 2>&1
echo "prof rc=$?"; tail -1 "$R/$OUT/hlds_bench_prof.log" | cut -c1-300
exit 0
