#!/bin/bash
# Copy a tools/gpu_r04_prof.sh run's results from gpurun_out/r04prof/ into profiles/ under the
# names tools/r04_table.py reads (bench log, kernel-trace stats, PMC counter CSVs, traffic.json).
set -eu
cd "$(dirname "$0")/.."
S=gpurun_out/r04prof
for d in $S/prof_*/; do
  t=$(basename $d); t=${t#prof_}
  cp $S/prof_$t.log profiles/r04prof_prof_$t.log
  cp $d/run_kernel_stats.csv profiles/r04prof_${t}_kernel_stats.csv
done
for d in $S/pmc_*/; do
  t=$(basename $d)
  cp $S/$t.log profiles/r04prof_$t.log
  cp $d/run_counter_collection.csv profiles/r04prof_${t}_counters.csv
done
for f in $S/bench_*.log; do [ -e "$f" ] && cp $f profiles/r04prof_$(basename $f); done
cp $S/traffic.json profiles/traffic.json
