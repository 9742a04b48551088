#!/bin/bash
# Copies the judged evidence of a tools/prof_round.sh run from gpurun_out/$1
# (scratch) into profiles/$1 (tracked): bench line, rocprofv3 --stats kernel
# summary, PMC digest and the render-kernel rows of each PMC pass.
set -e
R=${1:?round tag}
cd "$(dirname "$0")/.."
S=gpurun_out/$R; D=profiles/$R
mkdir -p $D
cp $S/bench.json $D/bench.json
cp $S/stats/bench_kernel_stats.csv $D/bench_kernel_stats.csv
cp $S/pmc_digest.json $D/pmc_digest.json
[ -f $S/bands_kernel_stats.csv ] && cp $S/bands_kernel_stats.csv $D/bands_kernel_stats.csv
for d in $S/pmc*/; do
  n=$(basename $d)
  f=$(ls $d/*counter_collection.csv)
  { head -1 $f; grep -E 'rt::(smallpt|whitted|queue)::' $f || true; } > $D/${n}_render_kernels.csv
done
ls -la $D
