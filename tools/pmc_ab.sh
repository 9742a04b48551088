#!/bin/bash
# PMC comparison of A/B variants (build_ab/<name>): counter passes per
# variant over one timed launch of tools/ab.py's workload.
# Usage: LIBS=a,b KERNEL=smallpt|whitted bash tools/pmc_ab.sh
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export REPS=1
mkdir -p gpurun_out/pmc_ab
SETS=(
 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU"
 "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_INT32 SQ_WAIT_INST_LDS"
 "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
)
for v in ${LIBS//,/ }; do
  export RT_HIP_LIB=$GRAFT_REPO_ROOT/build_ab/$v/librt_hip.so VARIANT=$v
  i=0
  for set in "${SETS[@]}"; do
    i=$((i+1))
    timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv --pmc $set -d gpurun_out/pmc_ab/$v/$i -o p \
        -- python3 tools/ab.py child > gpurun_out/pmc_ab/$v.$i.log 2>&1
  done
done
python3 tools/pmc_summary.py gpurun_out/pmc_ab
