#!/bin/bash
# PMC digest of the configs[4] (hierarchy) kernel: tools/c5_time.py under
# rocprofv3 --pmc, one pass per ';'-separated counter set in $SETS (default:
# instruction mix / lane utilisation / VALU issue, then waits and memory).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export SPP=${SPP:-4}
OUT=gpurun_out/pmc_c5
rm -rf $OUT && mkdir -p $OUT
SETS=${SETS:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE;SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SMEM SQ_INSTS_BRANCH"}
i=0
IFS=';' read -ra SETARR <<< "$SETS"
for set in "${SETARR[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc $set -d $OUT/pmc$i -o p \
      -- python3 tools/c5_time.py > $OUT/pmc$i.log 2>&1
done
python3 tools/pmc_digest.py $OUT > /dev/null
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob('gpurun_out/pmc_c5/pmc*/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r['Kernel_Name'][:60]][r['Counter_Name']] += float(r['Counter_Value'])
for k, v in agg.items():
    print(k, dict(v))
PY
