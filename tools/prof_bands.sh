#!/bin/bash
# rocprofv3 --kernel-trace --stats of one N-GPU row band rendered alone on one
# MI355X (tools/ab.py child, BAND=k/N, REPS+1 launches incl. the first), for
# N = 2, 4, 8.  Output: gpurun_out/$1/bands_kernel_stats.csv (one section per band).
set -e
R=${1:?round tag}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$R
mkdir -p $O
OUT=$O/bands_kernel_stats.csv
echo "# rocprofv3 --kernel-trace --stats of one N-GPU row band rendered alone on one MI355X (tools/ab.py child, BAND=k/N, 6 launches incl. the first); columns as bench_kernel_stats.csv" > $OUT
for b in 1/2 1/4 1/8; do
  tag=band${b%/*}of${b#*/}
  BAND=$b REPS=5 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag -o s \
      -- python3 tools/ab.py child > $O/$tag.log 2>&1
  echo "# $tag" >> $OUT
  cat $O/$tag/s_kernel_stats.csv >> $OUT
done
