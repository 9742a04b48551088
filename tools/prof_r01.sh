#!/bin/bash
# Round-1 evidence run on the GPU box: bench line, rocprofv3 kernel stats of
# the same bench command, and HBM traffic counters (one counter per pass).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r01
timeout -k 10 300 python3 bench.py > gpurun_out/r01/bench.json 2> gpurun_out/r01/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r01/stats -o bench \
    -- python3 bench.py --no-cpu > gpurun_out/r01/stats_bench.json 2> gpurun_out/r01/stats.err
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc $c -d gpurun_out/r01/pmc_$c -o p \
      -- python3 tools/prof_kernels.py --reps 1 > gpurun_out/r01/pmc_$c.log 2>&1
done
