#!/bin/bash
# Evidence run on the GPU box for round $1 (e.g. r01): the default bench line,
# a rocprofv3 --kernel-trace --stats summary of the same bench command, and
# PMC passes over the bench workload (one TCC counter per pass, as the
# MI355X HBM/rocprofv3 guide prescribes; SQ instruction-mix counters apart).
# Output: gpurun_out/$1/ ; tools/pmc_digest.py condenses it for profiles/$1/.
set -e
R=${1:?round tag}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$R
mkdir -p $O
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o bench \
    -- python3 bench.py --no-cpu --no-cornell-extra > $O/stats_bench.json 2> $O/stats.err
B="python3 bench.py --no-cpu --no-cornell-extra --steps 2 --warmup 1"
i=0
for set in FETCH_SIZE WRITE_SIZE \
    "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE" \
    "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc $set -d $O/pmc$i -o p \
      -- $B > $O/pmc$i.log 2>&1
done
python3 tools/pmc_digest.py $O > $O/pmc_digest.json
